"""Build the oracle's native checkers into oracle/_build/ (test infrastructure only; never
linked into the product).  Run by __graft_entry__.build() and `python -m oracle.build`.

  librocrand_words.so  rocRAND's own Philox4x32-10 on the host (oracle/rocrand_words.cpp)
"""
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
OUT_DIR = os.path.join(HERE, "_build")
ROCRAND_SRC = os.path.join(HERE, "rocrand_words.cpp")
ROCRAND_LIB = os.path.join(OUT_DIR, "librocrand_words.so")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")


def build(force=False, verbose=False):
    os.makedirs(OUT_DIR, exist_ok=True)
    if force or not os.path.exists(ROCRAND_LIB) or os.path.getmtime(ROCRAND_LIB) < os.path.getmtime(ROCRAND_SRC):
        # host code only: rocRAND's engine functions are __host__ __device__
        cmd = [HIPCC, "-O2", "-fPIC", "-shared", "-std=c++17", "-x", "c++", "-D__HIP_PLATFORM_AMD__",
               "-I/opt/rocm/include", "-o", ROCRAND_LIB, ROCRAND_SRC]
        if verbose:
            print(" ".join(cmd))
        subprocess.run(cmd, check=True)
    return ROCRAND_LIB


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
