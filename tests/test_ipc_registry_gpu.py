"""Process-wide IPC mappings: two communicators and an
osc window map the same peer device buffers; freeing one holder must leave
the others working bit-exactly (tests/ipc_share_worker.py)."""
import json
import os

import pytest

from test_coll_gpu import run_ranks

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
WORKER = os.path.join(ROOT, "tests", "ipc_share_worker.py")


@pytest.mark.parametrize("n", [2, 4])
def test_shared_mappings_survive_one_holder(n):
    outs = run_ranks(n, timeout=300, worker=WORKER, tag="ipc_share_n")
    failures = []
    for r, (rc, out) in enumerate(outs):
        lines = [json.loads(ln) for ln in out.splitlines() if ln.startswith("{")]
        bad = [ln for ln in lines if not ln["ok"]]
        if rc != 0 or bad or len(lines) < 5:
            failures.append((r, rc, bad[:3], out[-2000:]))
    assert not failures, failures
