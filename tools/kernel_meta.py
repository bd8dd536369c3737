#!/usr/bin/env python3
"""Code-object metadata (and optionally a disassembly digest) of every kernel in a built
gfx950 library:

    python tools/kernel_meta.py [lib.so] [--filter SUBSTR] [--json OUT] [--digest]

Per kernel: VGPRs, AGPRs, SGPRs, VGPR / SGPR spill counts, scratch per lane
(`.private_segment_fixed_size`), LDS (`.group_segment_fixed_size`), and with --digest a
hash of the kernel's instructions with addresses, branch offsets and PC-relative global
offsets stripped, so two
builds of the same source can be compared kernel by kernel (a refactor that must leave
the default kernels' code unchanged).  The data come from `llvm-readelf --notes` of the
code object unbundled from `.hip_fatbin` (AMDGPU metadata, msgpack rendered as YAML)."""
import hashlib
import json
import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
FIELDS = {".vgpr_count": "vgpr", ".agpr_count": "agpr", ".sgpr_count": "sgpr",
          ".vgpr_spill_count": "vgpr_spill", ".sgpr_spill_count": "sgpr_spill",
          ".private_segment_fixed_size": "scratch_B", ".group_segment_fixed_size": "lds_B"}


def code_objects(lib, td):
    """The gfx950 code object of every translation unit: .hip_fatbin holds one offload bundle
    per TU (hedge_env.hip, vecnorm.hip, analytics.hip), each unbundled on its own."""
    fb = os.path.join(td, "fb.bin")
    subprocess.run(["objcopy", "-O", "binary", "--only-section=.hip_fatbin", lib, fb], check=True)
    data = open(fb, "rb").read()
    magic = b"__CLANG_OFFLOAD_BUNDLE__"
    starts = [m.start() for m in re.finditer(re.escape(magic), data)]
    cos = []
    for k, a in enumerate(starts):
        b = starts[k + 1] if k + 1 < len(starts) else len(data)
        part, co = os.path.join(td, "b%d.bin" % k), os.path.join(td, "co%d.o" % k)
        with open(part, "wb") as fh:
            fh.write(data[a:b])
        r = subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={part}",
                            "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}"], capture_output=True)
        if r.returncode == 0 and os.path.getsize(co) > 0:
            cos.append(co)
    return cos


def metadata(co):
    txt = subprocess.run([f"{LLVM}/llvm-readelf", "--notes", co], check=True, capture_output=True,
                         text=True).stdout
    lines = txt.split("\n")
    st = next(i for i, l in enumerate(lines) if l.strip() == "amdhsa.kernels:")
    # each kernel is one YAML map: "  - .first_key:" at the kernel list's indentation
    ind = re.match(r"(\s*)- ", lines[st + 1]).group(1)
    maps, cur = [], None
    for line in lines[st + 1:]:
        if line.startswith(ind + "- "):
            cur = {}
            maps.append(cur)
        elif line and not line.startswith(ind + " "):
            break
        if cur is None or not (line.startswith(ind + "- .") or line.startswith(ind + "  .")):
            continue  # the kernel's own keys only (not the nested .args entries)
        m = re.match(r"\s*-?\s*(\.[a-z_]+):\s+(.*)$", line)
        if m:
            cur[m.group(1)] = m.group(2).strip()
    out = {}
    for d in maps:
        sym = d.get(".symbol", "?")
        sym = sym[:-3] if sym.endswith(".kd") else sym
        out[sym] = {f: int(d[k]) if k in d else None for k, f in FIELDS.items()}
    return out


def digests(co):
    dis = subprocess.run([f"{LLVM}/llvm-objdump", "-d", "--no-show-raw-insn", co], check=True,
                         capture_output=True, text=True).stdout.split("\n")
    res, name, h, n = {}, None, None, 0
    recent = []   # the last two opcodes: PC-relative offsets follow s_getpc_b64
    for l in dis:
        if l.endswith(">:"):
            if name:
                res[name] = (h.hexdigest()[:16], n)
            name, h, n, recent = l.split("<")[1].rstrip(">:"), hashlib.sha256(), 0, []
            continue
        if name is None:
            continue
        m = re.match(r"\s+(\w+)\s*(.*?)\s*(//.*)?$", l)
        if not m or not m.group(1):
            continue
        ops = re.sub(r"<[^>]*>", "", m.group(2))
        if m.group(1).startswith("s_cbranch") or m.group(1) == "s_branch":
            ops = ""
        if m.group(1) in ("s_add_u32", "s_addc_u32") and "s_getpc_b64" in recent:
            ops = re.sub(r"0x[0-9a-f]+", "REL", ops)   # a global's offset: moves with the layout
        recent = (recent + [m.group(1)])[-2:]
        h.update((m.group(1) + " " + ops + "\n").encode())
        n += 1
    if name:
        res[name] = (h.hexdigest()[:16], n)
    return res


def main(argv):
    lib = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "cantorrl_amd", "lib", "libhedgeenv.so")
    flt, js, dig = None, None, False
    args = list(argv)
    while args:
        a = args.pop(0)
        if a == "--filter":
            flt = args.pop(0)
        elif a == "--json":
            js = args.pop(0)
        elif a == "--digest":
            dig = True
        else:
            lib = a
    with tempfile.TemporaryDirectory() as td:
        meta, dg = {}, {}
        for co in code_objects(lib, td):
            meta.update(metadata(co))
            if dig:
                dg.update(digests(co))
    rows = []
    for sym in sorted(meta):
        if flt and flt not in sym:
            continue
        r = dict(kernel=sym, **meta[sym])
        if dig:
            r["digest"], r["n_insts"] = dg.get(sym, (None, None))
        rows.append(r)
    for r in rows:
        print(json.dumps(r))
    if js:
        with open(js, "w") as f:
            json.dump(rows, f, indent=1)


if __name__ == "__main__":
    main(sys.argv[1:])
