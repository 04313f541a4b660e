import time, torch, os, sys
sys.path.insert(0, os.getcwd())
from evolutionarydistributedtraining_amd import checkpoint
from evolutionarydistributedtraining_amd.layouts import qwen2p5_7b_body
lay = qwen2p5_7b_body(); P = lay.total
x = torch.empty(P, dtype=torch.bfloat16, device="cuda")
x.fill_(0.5)
torch.cuda.synchronize()
for i in range(2):
    t0 = time.perf_counter(); h = checkpoint._host_copy(x); t1 = time.perf_counter()
    print(f"host copy {i}: {t1-t0:.3f} s", flush=True)
hdr = checkpoint._header_bytes(lay, lay.names, x.dtype, None)
os.makedirs("/tmp/wp", exist_ok=True)
for th in (1, 4, 16):
    t0 = time.perf_counter(); checkpoint._write_file(f"/tmp/wp/f{th}.safetensors", hdr, h, threads=th); t1 = time.perf_counter()
    print(f"write threads {th}: {t1-t0:.3f} s = {2*P/(t1-t0)/1e9:.2f} GB/s", flush=True)
    os.remove(f"/tmp/wp/f{th}.safetensors")
