"""Multi-process parity of the xGMI collectives against the oracle.

N ranks (one process each) run tests/coll_worker.py.  On a one-GPU box all
ranks share cuda:0: the IPC handles, flags, barriers, ring ownership and
operand order are exercised exactly as across GPUs (peer memory is then the
same device's memory, so only the link bandwidth differs).  On a multi-GPU
box rank r uses device r.
"""
import json
import os
import socket
import subprocess
import sys
import signal
import time

import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
WORKER = os.path.join(ROOT, "tests", "coll_worker.py")


def free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def run_ranks(n, timeout=600, extra_env=None, worker=WORKER, tag="n"):
    ngpu = torch.cuda.device_count()
    if "GRAFT_REPO_ROOT" in os.environ and "COLL_LOG_DIR" not in os.environ:
        # on the gpurun box: per-rank progress files under gpurun_out/ (a hang
        # names its case, and the progress keeps the silence watchdog off)
        os.environ["COLL_LOG_DIR"] = os.path.join(os.environ["GRAFT_REPO_ROOT"], "gpurun_out",
                                                  "coll_logs")
    port = free_port()
    logdir = os.environ.get("COLL_LOG_DIR")
    if logdir:
        os.makedirs(logdir, exist_ok=True)
    procs, files = [], []
    for r in range(n):
        env = dict(os.environ)
        env.update({"RANK": str(r), "WORLD_SIZE": str(n), "MASTER_ADDR": "127.0.0.1",
                    "MASTER_PORT": str(port), "LOCAL_RANK": str(r),
                    "OMPI_AMD_DEVICE": str(r % ngpu if ngpu >= n else 0)})
        # the HSA IPC mode is NOT forced here: the ranks run under whatever
        # the environment gives bench.py's N>1 leg and an mpirun job (the
        # library's load-time default when unset); each
        # worker reports the mode it ran under (coll_worker.py "ipc_mode")
        env.update(extra_env or {})
        # raw per-rank output (library diagnostics on stderr) goes straight to
        # a file, so that it survives a run killed at its time limit
        path = os.path.join(logdir, f"raw_{tag}{n}_rank{r}.txt") if logdir else None
        f = open(path, "w+") if path else subprocess.PIPE
        files.append(f)
        procs.append(subprocess.Popen([sys.executable, worker], env=env, stdout=f,
                                      stderr=subprocess.STDOUT, text=True))
    outs = []
    try:
        for p, f in zip(procs, files):
            out, _ = p.communicate(timeout=timeout)
            if f is not subprocess.PIPE:
                f.seek(0)
                out = f.read()
                f.close()
            outs.append((p.returncode, out))
    finally:
        alive = [p for p in procs if p.poll() is None]
        if alive and (extra_env or {}).get("OMPI_AMD_BACKTRACE", os.environ.get("OMPI_AMD_BACKTRACE")) == "1":
            for p in alive:  # each hung rank prints its Python stack, then its native one
                os.kill(p.pid, signal.SIGUSR1)
            time.sleep(2)
            for p in alive:
                os.kill(p.pid, signal.SIGUSR2)
            time.sleep(3)
        for p in alive:
            if p.poll() is None:
                p.kill()
    return outs


@pytest.mark.parametrize("n", [2, 4, 3, 8])
def test_collectives_parity(n):
    env = {"COLL_BIG": str(1 << 20)} if n == 8 else None
    outs = run_ranks(n, extra_env=env)
    failures = []
    for r, (rc, out) in enumerate(outs):
        lines = [json.loads(ln) for ln in out.splitlines() if ln.startswith("{")]
        bad = [ln for ln in lines if not ln["ok"]]
        mode = [ln for ln in lines if ln["case"] == "ipc_mode"]
        # the dmabuf IPC mode (HSA_ENABLE_IPC_MODE_LEGACY=0) is the one the
        # product runs under; the worker reports what it got
        if mode and mode[0]["legacy"] != 0:
            bad.append(mode[0])
        if rc != 0 or bad or not lines:
            failures.append((r, rc, bad[:3], out[-1500:] if not lines or rc not in (0, 1) else ""))
    assert not failures, failures


def test_allreduce_headline_size_n8():
    """256 MiB fp32 SUM allreduce at N = 8 (BASELINE's headline point), all
    seven large-message schemes (four phased, three pipelined), every element
    exact (dataset E)."""
    outs = run_ranks(8, extra_env={"COLL_HEADLINE": str(64 << 20)})
    failures = []
    for r, (rc, out) in enumerate(outs):
        lines = [json.loads(ln) for ln in out.splitlines() if ln.startswith("{")]
        lines = [ln for ln in lines if ln["case"] != "ipc_mode"]
        bad = [ln for ln in lines if not ln["ok"]]
        if rc != 0 or bad or len(lines) != 7:
            failures.append((r, rc, bad[:3], out[-1500:]))
    assert not failures, failures


def test_allreduce_past_ipc_cap_n2():
    """A 1.12 GB fp32 SUM allreduce at N = 2 under every scheme, every
    element exact (dataset E): its input and result shadows together pass
    the 2 GiB - 4 MiB IPC allocation cap, so pull+push
    runs them as two allocations, push-gather's landing buffer grows to
    (N + 1) slots of half the vector, and push-land (whose 2N slots would
    pass the cap) falls back to push-gather on every rank alike (its
    pipelined launch too); the pipelined schemes beside them."""
    outs = run_ranks(2, extra_env={"COLL_HEADLINE": str(280_000_000)})
    failures = []
    for r, (rc, out) in enumerate(outs):
        lines = [json.loads(ln) for ln in out.splitlines() if ln.startswith("{")]
        lines = [ln for ln in lines if ln["case"] != "ipc_mode"]
        bad = [ln for ln in lines if not ln["ok"]]
        if rc != 0 or bad or len(lines) != 7:
            failures.append((r, rc, bad[:3], out[-1500:]))
    assert not failures, failures


def test_waits_without_host_marks_n3():
    """The library's waits with host-observed completion marks off
    (OMPI_AMD_HOST_MARKS=0: blocking syncs, request and plan waits on events
    only): nonblocking and persistent allreduces, the
    pipelined nonblocking case and the nonblocking rsb / allgather / bcast
    stay exact against the oracle."""
    cases = ("iallreduce_mixed,iallreduce_many_outstanding,persistent_small,persistent_big,"
             "pipelined_nonblocking,nonblocking_rsb_ag_bcast,ar_sum_f32_big")
    outs = run_ranks(3, extra_env={"OMPI_AMD_HOST_MARKS": "0", "COLL_CASES": cases}, tag="nomarks_n")
    failures = []
    for r, (rc, out) in enumerate(outs):
        lines = [json.loads(ln) for ln in out.splitlines() if ln.startswith("{")]
        lines = [ln for ln in lines if ln["case"] != "ipc_mode"]
        bad = [ln for ln in lines if not ln["ok"]]
        if rc != 0 or bad or len(lines) != 7:
            failures.append((r, rc, bad[:3], [ln["case"] for ln in lines], out[-1500:]))
    assert not failures, failures
