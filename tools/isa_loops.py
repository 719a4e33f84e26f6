#!/usr/bin/env python3
"""Loop map of one structured-kernel instance in the built library: disassembles the gfx950 code
object (llvm-objdump --offloading into a temp dir, then -d), finds the instance's function, and
lists every backward branch (a loop: target .. branch) with its instruction count and the scratch,
global and LDS memory instructions inside it -- where the register spills land relative to the
ADMM iteration loop.  Usage: python tools/isa_loops.py '<256, 3, 3, 1, 39' [lib.so] [min_len]"""
import os
import re
import shutil
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
want = sys.argv[1] if len(sys.argv) > 1 else "<256, 3, 3, 1, 39"
lib = os.path.abspath(sys.argv[2] if len(sys.argv) > 2 else os.path.join(os.path.dirname(__file__), "..",
                                                                         "intent-mpc_amd", "lib", "libimpc_qp.so"))
min_len = int(sys.argv[3]) if len(sys.argv) > 3 else 200
tmp = tempfile.mkdtemp()
try:
    src = os.path.join(tmp, os.path.basename(lib))
    shutil.copy(lib, src)
    subprocess.run([f"{LLVM}/llvm-objdump", "--offloading", src], check=True, capture_output=True, cwd=tmp)
    co = sorted(f for f in os.listdir(tmp) if "gfx950" in f)
    dis = "".join(subprocess.run([f"{LLVM}/llvm-objdump", "-d", "--demangle", "--no-show-raw-insn",
                                  os.path.join(tmp, c)], check=True, capture_output=True, text=True).stdout
                  for c in co)
finally:
    shutil.rmtree(tmp)

# functions: "<addr> <name>:" headers; instructions: "  <ws><mnemonic> ... // <addr>:" or "addr: insn"
funcs, cur = {}, None
for ln in dis.splitlines():
    m = re.match(r"^([0-9a-f]+) <(.*)>:$", ln)
    if m:
        cur = m.group(2)
        funcs[cur] = []
        continue
    if cur is None:
        continue
    m = re.match(r"^\s+(\S.*?)\s*//\s*([0-9A-Fa-f]+):", ln)
    if m:
        funcs[cur].append((int(m.group(2), 16), m.group(1)))
names = [n for n in funcs if "k_mpc_wave_group" in n and want in n]
if not names:
    sys.exit(f"no k_mpc_wave_group instance matching {want!r}")
name = names[0]
ins = funcs[name]
print(name[:160], len(ins), "instructions")
pos = {a: i for i, (a, _) in enumerate(ins)}
loops = []
for i, (a, t) in enumerate(ins):
    m = re.match(r"s_(cbranch_\w+|branch)\s+(-?\d+)", t)
    if not m:
        continue
    imm = int(m.group(2))
    if imm > 32767:
        imm -= 65536
    ta = a + 4 + 4 * imm  # SOPP simm16: dwords after the next instruction
    if ta < a and ta in pos:
        loops.append((pos[ta], i))


def kinds(lo, hi):
    c = {"scratch_ld": 0, "scratch_st": 0, "global_ld": 0, "global_st": 0, "ds": 0, "valu": 0, "salu": 0,
         "s_waitcnt": 0, "s_barrier": 0}
    for _, t in ins[lo:hi + 1]:
        op = t.split()[0]
        if op.startswith("scratch_load") or op.startswith("buffer_load"):
            c["scratch_ld"] += 1
        elif op.startswith("scratch_store") or op.startswith("buffer_store"):
            c["scratch_st"] += 1
        elif op.startswith("global_load") or op.startswith("flat_load"):
            c["global_ld"] += 1
        elif op.startswith(("global_store", "global_atomic", "flat_store", "flat_atomic")):
            c["global_st"] += 1
        elif op.startswith("ds_"):
            c["ds"] += 1
        elif op.startswith("s_waitcnt"):
            c["s_waitcnt"] += 1
        elif op.startswith("s_barrier"):
            c["s_barrier"] += 1
        elif op.startswith("v_"):
            c["valu"] += 1
        elif op.startswith("s_"):
            c["salu"] += 1
    return c


tot = kinds(0, len(ins) - 1)
print("whole function:", tot)
for lo, hi in sorted(loops, key=lambda x: x[1] - x[0], reverse=True):
    if hi - lo < min_len:
        continue
    print(f"loop {ins[lo][0]:#x}..{ins[hi][0]:#x} ({hi - lo + 1} instructions):", kinds(lo, hi))
