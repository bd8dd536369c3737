#!/usr/bin/env python3
"""Static instruction mix of the loops of one kernel in a built libhedgeenv.so:

    python tools/isa_loops.py [lib.so] [kernel-substring] [n_loops]

Extracts the gfx950 code object (objcopy + clang-offload-bundler), disassembles it and
prints, for the largest loops (backward branches), the counts per instruction class."""
import collections
import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
lib = sys.argv[1] if len(sys.argv) > 1 else os.path.join(os.path.dirname(__file__), "..", "cantorrl_amd", "lib",
                                                         "libhedgeenv.so")
kern = sys.argv[2] if len(sys.argv) > 2 else "lds_rollout_kernelILi1ELb0ELb1E"
nl = int(sys.argv[3]) if len(sys.argv) > 3 else 6
with tempfile.TemporaryDirectory() as td:
    fb, co = os.path.join(td, "fb.bin"), os.path.join(td, "co.o")
    subprocess.run(["objcopy", "-O", "binary", "--only-section=.hip_fatbin", lib, fb], check=True)
    subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={fb}",
                    "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}"], check=True)
    dis = subprocess.run([f"{LLVM}/llvm-objdump", "-d", "--no-show-raw-insn", co], check=True,
                         capture_output=True, text=True).stdout.split("\n")
st = [i for i, l in enumerate(dis) if l.endswith(">:") and kern in l][0]
name = dis[st].split("<")[1].rstrip(">:")
en = st + 1
while en < len(dis) and not dis[en].endswith(">:"):
    en += 1
ins, base = [], None
for l in dis[st + 1:en]:
    m = re.match(r"\s+(\w+)\s*(.*?)\s*//\s*([0-9A-F]+):?", l)
    if not m:
        continue
    a = int(m.group(3), 16)
    base = a if base is None else base
    t = re.search(re.escape(name) + r"\+0x([0-9a-f]+)>", l)
    ins.append((a - base, m.group(1), int(t.group(1), 16) if t else None))
off2i = {o: k for k, (o, _, _) in enumerate(ins)}
loops = sorted(((off2i[tg], i) for i, (o, op, tg) in enumerate(ins) if tg is not None and tg <= o and op.startswith("s_")
                and tg in off2i), key=lambda x: x[0] - x[1])


def cls(op):
    if op.startswith("v_"):
        if "f64" in op:
            return "v_f64"
        if op.split("_")[1] in ("exp", "log", "rcp", "rsq", "sqrt", "sin", "cos"):
            return "v_trans"
        return "v_other"
    if op.startswith("ds_"):
        return "ds"
    if op.startswith(("global_", "buffer_", "flat_")):
        return "vmem"
    if op == "s_waitcnt":
        return "wait"
    if op.startswith("s_cbranch_exec"):
        return "br_exec"
    return "s"


print(name, "instructions", len(ins))
for j, i in loops[:nl]:
    c = collections.Counter(cls(op) for _, op, _ in ins[j:i + 1])
    print(f"  loop [{ins[j][0]:#x},{ins[i][0]:#x}] n={i - j + 1}", dict(sorted(c.items())))
