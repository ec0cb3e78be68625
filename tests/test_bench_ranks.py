"""bench.py's own rank path on CPU: `python bench.py --gpus 2 --dry-run` starts two rank processes
through torch.distributed.run (gloo), each takes its fnv1a64(name) mod 2 shard of the named document
sets, the CPU oracle stands in for the engine, and rank 0 prints the node totals."""
import json
import os
import subprocess
import sys

import pytest

from conftest import ROOT


@pytest.mark.timeout(400) if hasattr(pytest.mark, "timeout") else (lambda f: f)
def test_bench_two_ranks_dry_run():
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--dry-run", "--docs", "30", "--updates", "12",
                        "--c2big-docs", "20", "--c4-docs", "150", "--steps", "2", "--warmup", "1"],
                       capture_output=True, text=True, timeout=380, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, r.stdout          # rank 0 only
    j = lines[0]
    assert j["n_gpus"] == 2 and j["scaling"] == "weak"
    assert j["config"]["docs_total"] == 60 and j["config"]["docs_per_gpu"] == 30
    assert j["config"]["updates_total"] == 60 * 12
    assert j["c2_100k"]["docs_total"] == 40
    assert j["c4"]["docs_total"] == 150 and set(j["c4"]) >= {"sv", "diff"}
    # single-process totals of the same named document sets
    sys.path.insert(0, ROOT)
    import numpy as np
    from tools import synth
    a, o, d = synth.text_updates_docs(np.arange(60), 12)
    assert j["config"]["bytes_in_total"] == len(a)
    a4, *_ = synth.text_states(150, seed=3)
    assert j["c4"]["bytes_in_total"] == len(a4)


def test_partition_matches_shard_of():
    import sys
    sys.path.insert(0, ROOT)
    from hocuspocus_amd.shard import shard_of
    from tools import synth
    for world in (2, 3, 8):
        parts = [set(synth.partition("c4-", 500, world, r).tolist()) for r in range(world)]
        assert sum(map(len, parts)) == 500 and set().union(*parts) == set(range(500))
        for r, p in enumerate(parts):
            assert all(shard_of(f"c4-{i}", world) == r for i in p)
