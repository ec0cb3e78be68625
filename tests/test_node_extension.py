"""The Node drop-in (packages/extension-gpu-merge): GpuMerge Extension hooks driven by a
mini Hocuspocus lifecycle (test/harness.js), mirroring the reference's own persistence
tests (SURVEY.md §8c semantic pins)."""
import os
import shutil
import subprocess

import pytest

from conftest import ROOT

PKG = os.path.join(ROOT, "packages", "extension-gpu-merge")
BUNDLE = "/opt/conda/share/jupyter/lab/static/3502.fbe0c610be82ba1360db.js"
needs_node = pytest.mark.skipif(shutil.which("node") is None or not os.path.exists(BUNDLE),
                                reason="node or the bundled yjs (test oracle) not present")


def run(mode):
    r = subprocess.run(["node", "--expose-gc", os.path.join(PKG, "test", "run.js"), f"--{mode}"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "passed" in r.stdout


@needs_node
def test_extension_hooks_cpu_double():
    run("cpu")


@needs_node
@pytest.mark.gpu
def test_extension_hooks_gpu_addon():
    assert os.path.exists(os.path.join(PKG, "build", "ygm_napi.node")), "N-API addon not built"
    run("gpu")
