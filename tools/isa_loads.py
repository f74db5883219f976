"""Memory-op schedule of one kernel in a HIP source (gfx950 ISA): which global loads issue back to
back and where the vmcnt waits fall -- the latency shape of a latency-bound kernel.

    python tools/isa_loads.py <file.hip> <kernel-name-substring> [max lines]
"""
import re
import subprocess
import sys

src, pat = sys.argv[1], sys.argv[2]
limit = int(sys.argv[3]) if len(sys.argv) > 3 else 150
cmd = ["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "-I/root/repo/include",
       "-mllvm", "-amdgpu-mfma-vgpr-form=1", "-x", "hip", "--cuda-device-only", "-S", src, "-o", "/tmp/_isa.s"]
subprocess.run(cmd, check=True, capture_output=True)
s = open("/tmp/_isa.s").read()
names = [m for m in re.findall(r"^(_Z\S*):", s, re.M) if pat in m]
if not names:
    sys.exit(f"no kernel matching {pat}")
name = names[0]
body = s[s.index(name + ":"):]
body = body[:body.index(".Lfunc_end")]
lines = [l.strip() for l in body.splitlines() if l.strip() and not l.strip().startswith((".", ";"))]
print(name, len(lines), "instructions")
keep = ("global_load", "global_store", "buffer_", "s_waitcnt vmcnt", "s_cbranch", "v_mfma", "s_barrier")
n = 0
for i, l in enumerate(lines):
    if l.startswith(keep):
        print(f"{i:5d} {l[:70]}")
        n += 1
        if n >= limit:
            break
