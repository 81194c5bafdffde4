"""Multi-process point-to-point and one-sided (§8f row 4)
tests on device buffers: N ranks run tests/p2p_osc_worker.py.  On a one-GPU
box all ranks share cuda:0 (IPC mappings, mailboxes, lock words and kernels
are exercised exactly as across GPUs; only the link differs)."""
import json
import os

import pytest

from test_coll_gpu import run_ranks

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
WORKER = os.path.join(ROOT, "tests", "p2p_osc_worker.py")


@pytest.mark.parametrize("n", [2, 3, 4, 8])
def test_p2p_osc_parity(n):
    outs = run_ranks(n, timeout=300, worker=WORKER, tag="p2p_osc_n")
    failures, first = [], []
    for r, (rc, out) in enumerate(outs):
        lines = [json.loads(ln) for ln in out.splitlines() if ln.startswith("{")]
        bad = [ln for ln in lines if not ln["ok"]]
        if rc != 0 or bad or not lines:
            failures.append((r, rc, bad[:4], out[-2000:] if not lines or rc not in (0, 1) else ""))
            if bad:  # every failing rank's first message, short (the rank that failed first shows)
                first.append(f"rank {r}: {bad[0]['case']}: {bad[0]['msg'][:300]}")
    assert not failures, ("\n".join(first), failures)


def test_osc_derived_accumulate_generic_offsets_n3():
    """The derived-datatype accumulates with the 64-bit typed-offset path
    (OMPI_AMD_OSC_DDT_FAST=0; the default takes 32-bit multiply-high
    divisors whenever the element counts fit): same oracle check."""
    outs = run_ranks(3, timeout=300, worker=WORKER, tag="p2p_osc_slowddt_n",
                     extra_env={"OMPI_AMD_OSC_DDT_FAST": "0",
                                "P2P_OSC_ONLY": "osc_accumulate_derived_datatypes"})
    for r, (rc, out) in enumerate(outs):
        lines = [json.loads(ln) for ln in out.splitlines() if ln.startswith("{")]
        assert rc == 0 and len(lines) == 1 and lines[0]["ok"], (r, rc, out[-2000:])
