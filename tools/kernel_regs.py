#!/usr/bin/env python3
"""Register / spill report of the structured kernel instances in the built library: extracts the
gfx950 code object (llvm-objdump --offloading, into a temp dir) and reads the AMDHSA metadata notes
(llvm-readelf --notes).  Usage: python tools/kernel_regs.py [lib.so] [name-filter]"""
import os
import re
import shutil
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
lib = os.path.abspath(sys.argv[1] if len(sys.argv) > 1 else os.path.join(os.path.dirname(__file__), "..",
                                                                         "intent-mpc_amd", "lib", "libimpc_qp.so"))
filt = sys.argv[2] if len(sys.argv) > 2 else "wave_group"
tmp = tempfile.mkdtemp()
try:
    src = os.path.join(tmp, os.path.basename(lib))
    shutil.copy(lib, src)  # objdump writes the bundles next to its input
    subprocess.run([f"{LLVM}/llvm-objdump", "--offloading", src], check=True, capture_output=True, cwd=tmp)
    co = sorted(f for f in os.listdir(tmp) if "gfx950" in f)  # one bundle per HIP translation unit
    out = "".join(subprocess.run([f"{LLVM}/llvm-readelf", "--notes", os.path.join(tmp, c)], check=True,
                                 capture_output=True, text=True).stdout for c in co)
finally:
    shutil.rmtree(tmp)
# each kernel's metadata map: fields in alphabetical order; '.name' sits among them
blocks, cur = [], {}
for ln in out.splitlines():
    m = re.match(r"\s+-?\s*\.(\w+):\s+(\S+)", ln)
    if not m:
        continue
    k, v = m.groups()
    if k == "agpr_count" and cur:  # the first field of each kernel's map (alphabetical)
        blocks.append(cur)
        cur = {}
    cur[k] = v
blocks.append(cur)
for b in blocks:
    nm = b.get("name", "")
    if filt in nm:
        print(f"{nm[:90]:90s} vgpr {b.get('vgpr_count')} agpr {b.get('agpr_count')} spill {b.get('vgpr_spill_count')} "
              f"scratch {b.get('private_segment_fixed_size')} lds {b.get('group_segment_fixed_size')}")
