"""The C-ABI boundary: library loads and exports every symbol include/ygm.h declares
(no compute calls: this runs without a GPU)."""
import ctypes
import os
import re

from conftest import ROOT

import hocuspocus_amd.engine as eng


def header_functions():
    src = open(os.path.join(ROOT, "include", "ygm.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(ygm_[a-z0-9_]+)\s*\(", src)))


def test_header_declares_the_boundary():
    fns = header_functions()
    for f in ("ygm_merge_v1", "ygm_diff_v1", "ygm_sv_from_update_v1", "ygm_open", "ygm_close"):
        assert f in fns
    assert set(fns) == set(eng.EXPORTS)


def test_library_exports_every_declared_symbol():
    L = ctypes.CDLL(eng.LIB_PATH)
    for f in header_functions():
        assert hasattr(L, f), f


def test_strerror_and_version_without_gpu():
    assert "malformed" in eng.strerror(eng.EMALFORMED)
    assert eng.lib().ygm_version().startswith(b"ygm")


def test_no_cpu_fallback_in_product():
    # the product package must never import the oracle (test infrastructure)
    pkg = os.path.join(ROOT, "hocuspocus_amd")
    for dp, _, fs in os.walk(pkg):
        for f in fs:
            if f.endswith((".py", ".cpp", ".hip", ".hpp", ".h", ".js", ".cc")):
                txt = open(os.path.join(dp, f), errors="ignore").read()
                assert "import oracle" not in txt and "liboracle" not in txt, f
