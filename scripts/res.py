"""Per-kernel VGPR / scratch / occupancy / LDS of a HIP source (gfx950)."""
import re, subprocess, sys
src = sys.argv[1]
pat = sys.argv[2] if len(sys.argv) > 2 else ""
out = subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC",
                      "-ffp-contract=off", "--offload-device-only", "-c", src, "-o", "/tmp/res.o",
                      "-Rpass-analysis=kernel-resource-usage"], capture_output=True, text=True).stderr
cur = None
rows = []
for line in out.splitlines():
    m = re.search(r"remark: (.*?): (.*)$", line)
    if not m:
        continue
    k, v = m.group(1).strip(), m.group(2).split(" [-R")[0].strip()
    if k == "Function Name":
        cur = {"name": v}
        rows.append(cur)
    elif cur is not None:
        cur[k] = v
for r in rows:
    if pat in r["name"]:
        print(f'{r.get("VGPRs","?"):>4} agpr {r.get("AGPRs","?"):>3} scr {r.get("ScratchSize [bytes/lane]","?"):>4} '
              f'occ {r.get("Occupancy [waves/SIMD]","?")} lds {r.get("LDS Size [bytes/block]","?"):>6}  {r["name"][:110]}')
