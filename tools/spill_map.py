#!/usr/bin/env python3
"""Where a kernel's VGPR spills are: builds a -gline-tables-only variant of libhedgeenv (same
flags otherwise), disassembles it with line info and counts the scratch instructions of the
kernels matching a substring per source line.

    python tools/spill_map.py [kernel-substring ...]   (default: the lds_rollout_kernels)
"""
import collections
import os
import re
import subprocess
import sys
import tempfile

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cantorrl_amd import build  # noqa: E402

LLVM = "/opt/rocm/lib/llvm/bin"


def main(subs):
    with tempfile.TemporaryDirectory() as td:
        so = build.build_variant(os.path.join(td, "dbg.so"), ["-gline-tables-only"])
        fb, co = os.path.join(td, "fb.bin"), os.path.join(td, "co.o")
        subprocess.run(["objcopy", "-O", "binary", "--only-section=.hip_fatbin", so, fb], check=True)
        subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={fb}",
                        "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}"], check=True)
        lines = subprocess.run([f"{LLVM}/llvm-objdump", "-d", "-l", "--no-show-raw-insn", co], check=True,
                               capture_output=True, text=True).stdout.split("\n")
    starts = [i for i, l in enumerate(lines) if l.endswith(">:")]
    for st in starts:
        name = lines[st]
        if not any(s in name for s in subs):
            continue
        en = st + 1
        while en < len(lines) and not lines[en].endswith(">:"):
            en += 1
        cur, cnt, tot = None, collections.Counter(), 0
        for l in lines[st:en]:
            m = re.match(r"; (/\S+):(\d+)", l)
            if m:
                cur = (os.path.basename(m.group(1)), int(m.group(2)))
                continue
            if "scratch_" in l:
                cnt[cur] += 1
                tot += 1
        print(name.split("<")[1].rstrip(">:")[:90], "scratch instructions:", tot)
        for k, v in cnt.most_common(25):
            print("    %s:%d  %d" % (k[0], k[1], v))


if __name__ == "__main__":
    main(sys.argv[1:] or ["lds_rollout_kernelILi1ELb1E", "lds_rollout_kernelILi2ELb1E"])
