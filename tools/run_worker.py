"""Run one multi-process worker (tests/coll_worker.py or tests/p2p_osc_worker.py)
at N ranks with extra environment, print every rank's failing lines.

    python tools/run_worker.py p2p_osc 8 P2P_OSC_CASES=a,b OSC_DIAG=1 STRESS_SEED=3000

Used for one-off GPU diagnostics; the suites use the same
launcher (tests/test_coll_gpu.py run_ranks)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))

from test_coll_gpu import run_ranks  # noqa: E402


def main():
    which, n = sys.argv[1], int(sys.argv[2])
    env = dict(kv.split("=", 1) for kv in sys.argv[3:])
    worker = os.path.join(ROOT, "tests", "p2p_osc_worker.py" if which == "p2p_osc" else "coll_worker.py")
    tag = env.pop("TAG", which + "_diag_n")
    outs = run_ranks(n, timeout=int(env.pop("TIMEOUT", "300")), worker=worker, tag=tag, extra_env=env)
    ok = True
    for r, (rc, out) in enumerate(outs):
        lines = [json.loads(ln) for ln in out.splitlines() if ln.startswith("{")]
        for ln in lines:
            if not ln.get("ok", True):
                ok = False
                print(json.dumps({"rank": r, "case": ln["case"], "msg": ln.get("msg", "")[:1500]}))
        if rc != 0 or not lines:
            ok = False
            print(json.dumps({"rank": r, "rc": rc, "tail": out[-1500:]}))
    print(json.dumps({"summary": "ok" if ok else "FAIL", "n": n, "env": env}))
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()
