"""Print per-kernel register usage / spills of one HIP source (gfx950 cross-compile)."""
import re
import subprocess
import sys

src = sys.argv[1]
extra = sys.argv[2:]
r = subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "-munsafe-fp-atomics",
                    "-I", "dl4ss_amd/csrc", *extra, "-c", src, "-o", "/tmp/kres.o",
                    "-Rpass-analysis=kernel-resource-usage"], capture_output=True, text=True)
cur = None
rows = {}
for line in r.stderr.splitlines():
    m = re.search(r"remark: +(\w[\w ]*?): (.*?) \[-Rpass", line)
    if not m:
        continue
    k, v = m.group(1).strip(), m.group(2).strip()
    if k == "Function Name" or k == "Name":
        cur = v
        rows[cur] = {}
    elif cur:
        rows[cur][k] = v
for name, d in rows.items():
    n = subprocess.run(["c++filt", name], capture_output=True, text=True).stdout.strip()
    n = n.replace("(anonymous namespace)::", "")
    print(f"{n[:70]:70s} V{d.get('VGPRs','?'):>4} A{d.get('AGPRs','?'):>3} "
          f"Sspill {d.get('SGPRs Spill','?'):>3} Vspill {d.get('VGPRs Spill','?'):>4} occ {d.get('Occupancy [waves/SIMD]','?')}")
if r.returncode:
    print(r.stderr[-3000:])
