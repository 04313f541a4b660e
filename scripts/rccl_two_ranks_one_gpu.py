"""Can RCCL run two ranks on ONE GPU (this pool's boxes have one)? Two processes, both on cuda:0,
torch.distributed "nccl": all_reduce, reduce_scatter, all_gather, all_to_all and a grouped p2p,
each checked. Prints one JSON line per rank. Launch:
    python scripts/rccl_two_ranks_one_gpu.py            (spawns the two ranks itself)
"""
import json
import os
import socket
import subprocess
import sys


def rank_main():
    import torch
    import torch.distributed as dist
    r, w = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=r, world_size=w, device_id=dev)
    out = {"rank": r}
    x = torch.full((1 << 20,), float(r + 1), device=dev)
    dist.all_reduce(x)
    out["all_reduce"] = bool((x == sum(range(1, w + 1))).all())
    inp = torch.arange(w * 4, dtype=torch.float32, device=dev) + 100 * r
    o = torch.empty(4, device=dev)
    dist.reduce_scatter_tensor(o, inp)
    want = sum(torch.arange(w * 4, dtype=torch.float32) + 100 * k for k in range(w))[r * 4:(r + 1) * 4]
    out["reduce_scatter"] = bool(torch.equal(o.cpu(), want))
    g = torch.empty(w * 4, device=dev)
    dist.all_gather_into_tensor(g, torch.full((4,), float(r), device=dev))
    out["all_gather"] = bool(torch.equal(g.cpu(), torch.arange(w).float().repeat_interleave(4)))
    a = torch.arange(w, dtype=torch.float32, device=dev) + 10 * r
    b = torch.empty(w, device=dev)
    dist.all_to_all_single(b, a)
    out["all_to_all"] = bool(torch.equal(b.cpu(), torch.tensor([10.0 * k + r for k in range(w)])))
    peer = 1 - r
    s, rv = torch.full((8,), float(r), device=dev), torch.empty(8, device=dev)
    reqs = dist.batch_isend_irecv([dist.P2POp(dist.isend, s, peer), dist.P2POp(dist.irecv, rv, peer)])
    for q in reqs:
        q.wait()
    out["p2p"] = bool((rv == float(peer)).all())
    torch.cuda.synchronize()
    dist.destroy_process_group()
    print(json.dumps(out), flush=True)


def main():
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    procs = []
    for r in range(2):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE="2", MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), EDT_RCCL_PROBE_RANK="1")
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)], env=env))
    rc = [p.wait(timeout=240) for p in procs]
    sys.exit(max(abs(c) for c in rc))


if __name__ == "__main__":
    rank_main() if os.environ.get("EDT_RCCL_PROBE_RANK") else main()
