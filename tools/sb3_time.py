"""Host-API timing (bench.sb3_api) of this tree or of another copy of the Python package.

    python tools/sb3_time.py [--pkg DIR] [--envs 2,256,65536] [--steps 504] [--out FILE]

--pkg DIR puts DIR first on sys.path, so `import cantorrl_amd` is that copy (e.g. the
round-4 host code snapshotted under tools/ab/r04_host) while the shared library stays this
tree's (CANTORRL_HEDGEENV_LIB): an A/B of the Python host path alone, same kernels.
"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pkg", default=None)
    ap.add_argument("--envs", default="2,256,65536")
    ap.add_argument("--steps", type=int, default=504)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    if a.pkg:
        sys.path.insert(0, os.path.abspath(a.pkg))
        os.environ.setdefault("CANTORRL_HEDGEENV_LIB", os.path.join(REPO, "cantorrl_amd", "lib", "libhedgeenv.so"))
    sys.path.insert(1 if a.pkg else 0, REPO)
    import torch
    import cantorrl_amd   # before bench, which puts REPO first on sys.path
    import bench
    from cantorrl_amd.vec_env import HedgingVecEnv, MONITOR_KEYWORDS
    from cantorrl_amd.env import HedgingEnv
    from cantorrl_amd.vec_normalize import DeviceVecNormalize
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    envs = tuple(int(x) for x in a.envs.split(","))
    res = bench.sb3_api(dev, (HedgingVecEnv, HedgingEnv, DeviceVecNormalize, MONITOR_KEYWORDS), envs, a.steps)
    res["package"] = os.path.dirname(os.path.abspath(cantorrl_amd.__file__))
    line = json.dumps(res)
    print(line, flush=True)
    if a.out:
        with open(a.out, "a") as fh:
            fh.write(line + "\n")


if __name__ == "__main__":
    main()
