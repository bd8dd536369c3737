"""Build the gfx950 libraries in-tree: cantorrl_amd/lib/libhedgeenv.so (the env) and
cantorrl_amd/lib/librbergomi.so (the rough-Bergomi data generator), plus the host-only
CPython module cantorrl_amd/lib/_info_rows*.so (a step's SB3 info dicts, csrc/info_rows.c).

    python -m cantorrl_amd.build [--force]

Flags that matter for parity with the NumPy reference:
  -ffp-contract=off                       no a*b+c -> fma contraction
  -fhip-fp32-correctly-rounded-divide-sqrt  IEEE f32 '/' and sqrtf
  -fno-gpu-flush-denormals-to-zero        keep f32 denormals
"""
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
SRC = os.path.join(HERE, "csrc", "hedge_env.hip")
DEPS = [SRC, os.path.join(HERE, "csrc", "he_math.h"), os.path.join(REPO, "include", "hedge_env.h")]
OUT = os.path.join(HERE, "lib", "libhedgeenv.so")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("CANTORRL_ARCH", "gfx950")

FLAGS = [
    f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-shared",
    "-ffp-contract=off", "-fhip-fp32-correctly-rounded-divide-sqrt",
    "-fno-gpu-flush-denormals-to-zero", "-Wall", "-Wno-unused-function",
]
# hedge_env.hip only: MachineLICM hoists every f64 polynomial constant of the market
# code (Box-Muller, exp, marks, greeks) out of the block loops into VGPR pairs, which
# then spill (lds_rollout_kernel: 168 VGPRs + 236 B/lane of scratch; without it 80
# VGPRs, no scratch).  Rematerialising them at the use is cheaper than scratch.
# -phi-node-folding-threshold=8: SimplifyCFG otherwise leaves the autoreset of the LDS
# reward wave (a dozen selects on `term`, with the episode summaries) as an if/else,
# whose CFG merges cost waitcnt drains and, there, scratch.
ENV_FLAGS = ["-mllvm", "-disable-machine-licm", "-mllvm", "-phi-node-folding-threshold=8"]


RB_SRC = os.path.join(HERE, "csrc", "rbergomi.hip")
RB_DEPS = [RB_SRC, os.path.join(HERE, "csrc", "he_math.h"), os.path.join(REPO, "include", "rbergomi.h")]
RB_OUT = os.path.join(HERE, "lib", "librbergomi.so")
VN_SRC = os.path.join(HERE, "csrc", "vecnorm.hip")
AN_SRC = os.path.join(HERE, "csrc", "analytics.hip")
DEPS = DEPS + [VN_SRC, AN_SRC, os.path.join(HERE, "csrc", "vn_moments.h")]
TARGETS = [([SRC, VN_SRC, AN_SRC], DEPS, OUT, ENV_FLAGS), ([RB_SRC], RB_DEPS, RB_OUT, [])]


# host-only: the CPython module that builds a step's SB3 info dicts (csrc/info_rows.c)
import sysconfig  # noqa: E402
ROWS_SRC = os.path.join(HERE, "csrc", "info_rows.c")
ROWS_OUT = os.path.join(HERE, "lib", "_info_rows" + sysconfig.get_config_var("EXT_SUFFIX"))
ROWS_CMD = [os.environ.get("CC", "gcc"), "-O2", "-shared", "-fPIC", "-Wall", "-Werror",
            "-I" + sysconfig.get_paths()["include"]]


def needs_build(out=OUT, deps=DEPS):
    if not os.path.exists(out):
        return True
    t = os.path.getmtime(out)
    return any(os.path.getmtime(d) > t for d in deps)


def build(force=False, verbose=False):
    """Build every library that is missing or older than its sources; returns the env's."""
    for srcs, deps, out, extra in TARGETS:
        if not force and not needs_build(out, deps):
            continue
        os.makedirs(os.path.dirname(out), exist_ok=True)
        tmp = out + ".tmp"
        cmd = [HIPCC, *FLAGS, *extra, "-o", tmp, *srcs]
        if verbose:
            print(" ".join(cmd))
        subprocess.run(cmd, check=True)
        os.replace(tmp, out)
    if force or needs_build(ROWS_OUT, [ROWS_SRC]):
        tmp = ROWS_OUT + ".tmp"
        cmd = [*ROWS_CMD, "-o", tmp, ROWS_SRC]
        if verbose:
            print(" ".join(cmd))
        subprocess.run(cmd, check=True)
        os.replace(tmp, ROWS_OUT)
    return OUT


def build_variant(out, extra_flags):
    """Diagnostic / A-B builds (e.g. -DHE_TIMING) outside the package directory."""
    os.makedirs(os.path.dirname(os.path.abspath(out)), exist_ok=True)
    subprocess.run([HIPCC, *FLAGS, *ENV_FLAGS, *extra_flags, "-o", out, SRC, VN_SRC, AN_SRC], check=True)
    return out


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
