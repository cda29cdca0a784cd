"""Dev tool: per-kernel register / spill summary of csrc/alipmpc.hip for gfx950 (hipcc resource remarks)."""
import re
import subprocess
import sys
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.environ.get("REGS_SRC") or os.path.join(ROOT, "mujoco-lip-mpc-simulation_amd", "csrc", "alipmpc.hip")
cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-mllvm", "-disable-machine-licm",
       "-Wno-unused-value", "--cuda-device-only", "-c", "-o", "/tmp/alipmpc_regs.o", SRC,
       "-Rpass-analysis=kernel-resource-usage"] + sys.argv[1:]
out = subprocess.run(cmd, capture_output=True, text=True, cwd="/tmp").stderr
cur = None
rows = {}
for line in out.splitlines():
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        cur = m.group(1)
        rows[cur] = {}
        continue
    m = re.search(r"remark:\s+([A-Za-z ]+?)(?: \[bytes/lane\]| \[waves/SIMD\])?: (\d+)", line)
    if m and cur:
        rows[cur][m.group(1).strip()] = int(m.group(2))
for k, v in rows.items():
    print(f"{k:50s} vgpr={v.get('VGPRs')} agpr={v.get('AGPRs')} sgpr={v.get('SGPRs')} scratch={v.get('ScratchSize')} "
          f"vspill={v.get('VGPRs Spill')} sspill={v.get('SGPRs Spill')} occ={v.get('Occupancy')} lds={v.get('LDS Size')}")
if not rows:
    print(out[-3000:])
