"""Does torch.profiler (Kineto over the ROCm tracer) see the HIP library's own launches? One outer
step and one pair merge at a small size under the profiler; prints the device kernels it recorded."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from evolutionarydistributedtraining_amd import ops  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    P, K = 1 << 22, 8
    theta = torch.randn(P, device=dev)
    workers = [torch.randn(P, device=dev) for _ in range(K)]
    mom = torch.zeros(P, device=dev)
    ops.outer_step(theta, workers, mom, True, 0.7, 0.9, True)
    torch.cuda.synchronize()
    from torch.profiler import ProfilerActivity, profile
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA]) as prof:
        ops.outer_step(theta, workers, mom, True, 0.7, 0.9, True)
        torch.cuda.synchronize()
    rows = []
    for e in prof.events():
        if e.device_type == torch.autograd.DeviceType.CUDA:
            rows.append({"name": e.name[:120], "us": round(e.device_time, 2) if hasattr(e, "device_time") else None})
    print(json.dumps({"device_events": rows}, indent=1))


if __name__ == "__main__":
    main()
