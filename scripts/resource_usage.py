"""Per-kernel register / occupancy / spill table of one translation unit, from the compiler's
-Rpass-analysis=kernel-resource-usage remarks (no GPU needed).

    python scripts/resource_usage.py evolutionarydistributedtraining_amd/csrc/edt_slerp.hip [filter]
"""
import re
import subprocess
import sys

ROOT = __file__.rsplit("/scripts/", 1)[0]


def main():
    src = sys.argv[1]
    flt = sys.argv[2] if len(sys.argv) > 2 else ""
    cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off", "-fPIC",
           "--cuda-device-only", "-c", "-I", f"{ROOT}/include", "-I", f"{ROOT}/evolutionarydistributedtraining_amd/csrc",
           src, "-o", "/tmp/_ru.o", "-Rpass-analysis=kernel-resource-usage"]
    out = subprocess.run(cmd, capture_output=True, text=True).stderr
    cur, rows = None, []
    for line in out.splitlines():
        m = re.search(r"remark: (.*?) \[-Rpass", line)
        if not m:
            continue
        t = m.group(1).strip()
        if t.startswith("Function Name:"):
            cur = {"name": t.split(":", 1)[1].strip()}
            rows.append(cur)
        elif cur is not None and ":" in t:
            k, v = t.split(":", 1)
            cur[k.strip()] = v.strip()
    dem = subprocess.run(["c++filt"], input="\n".join(r["name"] for r in rows), capture_output=True, text=True).stdout
    for r, d in zip(rows, dem.splitlines()):
        d = d.replace("(anonymous namespace)::", "")
        if flt and flt not in d:
            continue
        name = d.split("(")[0][:110]
        print(f"{r.get('VGPRs', '?'):>4} vgpr  occ {r.get('Occupancy [waves/SIMD]', '?'):>2}  "
              f"spill {r.get('VGPRs Spill', '?')}/{r.get('SGPRs Spill', '?')}  lds {r.get('LDS Size [bytes/block]', '?'):>5}  {name}")


if __name__ == "__main__":
    main()
