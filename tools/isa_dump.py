#!/usr/bin/env python3
"""Disassembly of libhedgeenv with source lines (a -gline-tables-only build of this tree, same
flags otherwise) -> /tmp/he_dis.txt, and the per-step instruction count and source-line
breakdown between consecutive occurrences of a marker instruction in one kernel:

    python tools/isa_dump.py [kernel-substring] [marker-mnemonic] [which-occurrence]

Default: the headline kernel (lds_rollout_kernel<GBM, no book, lean>), v_log_f32 (one per obs
stepper step), all occurrences."""
import collections
import os
import re
import subprocess
import sys
import tempfile

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cantorrl_amd import build  # noqa: E402

LLVM = "/opt/rocm/lib/llvm/bin"
OUT = "/tmp/he_dis.txt"


def dump():
    with tempfile.TemporaryDirectory() as td:
        so = build.build_variant(os.path.join(td, "dbg.so"), ["-gline-tables-only"])
        fb, co = os.path.join(td, "fb.bin"), os.path.join(td, "co.o")
        subprocess.run(["objcopy", "-O", "binary", "--only-section=.hip_fatbin", so, fb], check=True)
        subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={fb}",
                        "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}"], check=True)
        txt = subprocess.run([f"{LLVM}/llvm-objdump", "-d", "-l", "--no-show-raw-insn", co], check=True,
                             capture_output=True, text=True).stdout
    open(OUT, "w").write(txt)


def main():
    kern = sys.argv[1] if len(sys.argv) > 1 else "lds_rollout_kernelILi1ELb0ELb1E"
    mark = sys.argv[2] if len(sys.argv) > 2 else "v_log_f32"
    if not os.path.exists(OUT) or os.environ.get("REDUMP"):
        dump()
    lines = open(OUT).read().split("\n")
    st = [i for i, l in enumerate(lines) if l.endswith(">:") and kern in l][0]
    en = st + 1
    while en < len(lines) and not lines[en].endswith(">:"):
        en += 1
    seg = lines[st:en]
    idx = [i for i, l in enumerate(seg) if re.match(r"\s+" + mark + r"(_e32|_e64)?\s", l)]
    print("occurrences of", mark, len(idx))
    for a, b in zip(idx, idx[1:]):
        n = sum(1 for l in seg[a:b] if re.match(r"\s+\w", l))
        print(f"  [{a}, {b}) {n} instructions")
    if len(sys.argv) > 3:
        k = int(sys.argv[3])
        a, b = idx[k], idx[k + 1]
        c, src, cur = collections.Counter(), collections.Counter(), None
        for l in seg[a:b]:
            m = re.match(r"; (/\S+):(\d+)", l)
            if m:
                cur = m.group(1).split("/")[-1] + ":" + m.group(2)
                continue
            m = re.match(r"\s+(\w+)", l)
            if m:
                c[m.group(1)] += 1
                src[cur] += 1
        print(sorted(c.items(), key=lambda x: -x[1])[:40])
        for kk, v in src.most_common(45):
            print(f"  {v:4d} {kk}")


if __name__ == "__main__":
    main()
