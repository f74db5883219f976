"""Per-kernel register / LDS / occupancy summary of one HIP source (hipcc resource remarks).

    python tools/kres.py <file.hip> [extra hipcc flags...]
"""
import re, subprocess, sys

src, extra = sys.argv[1], sys.argv[2:]
cmd = ["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950", "-I/root/repo/include",
       "-x", "hip", "-c", src, "-o", "/tmp/_kres.o", "-Rpass-analysis=kernel-resource-usage"] + extra
out = subprocess.run(cmd, capture_output=True, text=True).stderr
cur = None
rows = {}
for line in out.splitlines():
    m = re.search(r"remark:\s+(.*?)\s+\[-Rpass", line)
    if not m:
        continue
    txt = m.group(1)
    if txt.startswith("Function Name:"):
        cur = txt.split(":", 1)[1].strip()
        rows[cur] = {}
    elif cur and ":" in txt:
        k, v = txt.split(":", 1)
        rows[cur][k.strip()] = v.strip()
for name, r in rows.items():
    short = re.sub(r"^_ZN3gpk(12_GLOBAL__N_1)?\d+", "", name)[:60]
    print(f"{short:60s} V {r.get('VGPRs','?'):>4} A {r.get('AGPRs','?'):>4} scr {r.get('ScratchSize [bytes/lane]','?'):>4} "
          f"LDS {r.get('LDS Size [bytes/block]','?'):>6} occ {r.get('Occupancy [waves/SIMD]','?')}")
