"""The bench's point-to-point / one-sided rows alone (ompi_amd/coll_bench.py
_p2p_osc_rows), N ranks on this box's GPUs (shared when fewer), for the
latency-cliff study of DESIGN.md §6.6:

    python tools/p2p_osc_rows.py N [OUT.json]

Each rank is a child process (gloo for the host-side timing collectives);
env passes through, so GPU_MAX_HW_QUEUES or OMPI_AMD_* can be varied."""
import json
import os
import socket
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def rank_main():
    sys.path.insert(0, ROOT)
    import torch
    import torch.distributed as dist
    from ompi_amd import coll, coll_bench
    from ompi_amd import op as mop
    rank, n = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    ngpu = torch.cuda.device_count()
    dev = rank % ngpu if ngpu >= n else 0
    torch.cuda.set_device(dev)
    dist.init_process_group("gloo", rank=rank, world_size=n)
    comm = coll.Communicator.from_torch_distributed(device=dev)
    if os.environ.get("ROWS_OWN_STREAM") == "1":
        comm.set_param("own_stream", 1)
    pre = os.environ.get("ROWS_PRE", "")
    if pre:
        # a collective first, as the bench's allreduce legs run before these
        # rows: iar_big / ar_big a (non)blocking allreduce past the zero-copy
        # size (a landing growth: queued at post / at the call), iar_small a
        # staged one (no growth)
        x = torch.ones((16 << 20) if pre.endswith("big") else 1024, device="cuda")
        y = torch.empty_like(x)
        torch.cuda.synchronize()
        for kind in pre.split("+")[0].split(","):  # e.g. ar,iar_big: a blocking call, then a nonblocking one
            if kind.startswith("iar"):
                comm.iallreduce(x, y, x.numel(), mop.MPI_FLOAT, mop.MPI_SUM).wait()
            elif kind.startswith("pers"):  # a persistent plan: init, two starts, free
                pl = comm.allreduce_init(x, y, x.numel(), mop.MPI_FLOAT, mop.MPI_SUM)
                for _ in range(2):
                    pl.start()
                    pl.wait()
                pl.free()
            elif kind.startswith("scan"):
                comm.scan(x, y, x.numel(), mop.MPI_FLOAT, mop.MPI_SUM)
            elif kind.startswith("auto"):  # autotuned blocking calls (the bench's rows run with it on)
                comm.set_param("autotune", 1)
                for _ in range(40):
                    comm.allreduce(x, y, x.numel(), mop.MPI_FLOAT, mop.MPI_SUM)
            else:
                comm.allreduce(x, y, x.numel(), mop.MPI_FLOAT, mop.MPI_SUM)
        torch.cuda.synchronize()
    res = coll_bench._p2p_osc_rows(comm, dist, torch, mop, n, rank, "cpu")
    res["pre"] = pre
    res["deferred_growths"] = comm.get_param("landing_deferred_growths")
    res["landing_bytes"] = comm.get_param("landing_bytes")
    res["ipc_live"] = comm.get_param("ipc_live")
    res["landing_retired"] = comm.get_param("landing_retired")
    if rank == 0:
        print(json.dumps({"ranks": n, "gpus": ngpu, "hw_queues": os.environ.get("GPU_MAX_HW_QUEUES", "default"),
                          "own_stream": os.environ.get("ROWS_OWN_STREAM", "0"), **res}), flush=True)
    comm.free()
    dist.destroy_process_group()


def main():
    n = int(sys.argv[1])
    out = sys.argv[2] if len(sys.argv) > 2 else None
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(n), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), ROWS_CHILD="1")
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)], env=env,
                                      stdout=subprocess.PIPE if r == 0 else subprocess.DEVNULL, text=True))
    line = procs[0].communicate(timeout=600)[0]
    rc = max(p.wait(timeout=600) for p in procs)
    if out:
        with open(out, "a") as f:
            f.write(line)
    print(line, end="")
    sys.exit(rc)


if __name__ == "__main__":
    rank_main() if os.environ.get("ROWS_CHILD") else main()
