"""Dev probe (tooling): ygm_sync_step2_v1 on a few fixture rows with YGM_DEBUG tracing."""
import os, sys
os.environ["YGM_DEBUG"] = "1"
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))), "tests"))
from test_step2 import rows
from hocuspocus_amd import Engine
r = rows()
for n in (1, 3, 50, len(r)):
    with Engine(0, compat135=True) as e:
        try:
            res = e.sync_step2_batch([u for u, *_ in r[:n]], [sv for _, sv, *_ in r[:n]])
            bad = sum(1 for (u, sv, exp, _), g in zip(r[:n], res) if (exp is None and g[0] != 4) or (exp is not None and g != (0, exp)))
            print(n, "ok, mismatches", bad, flush=True)
        except Exception as ex:
            print(n, "failed", ex, flush=True)
            snaps = e.snapshot_batch([u for u, *_ in r[:n]])
            print("  snapshot statuses", sorted(set(s for s, _ in snaps)), flush=True)
