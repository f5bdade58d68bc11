"""Build another libregnn_hip.so variant with extra compiler flags (A/B of kernel variants and the
phase-instrumented build; loaded on the GPU box through REGNN_LIB, tools/ab_lib.sh).
usage: python tools/build_variant.py NAME [-DFLAG ...]   -> ab/libregnn_NAME.so"""
import concurrent.futures as cf
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "re-gnn_amd"))
from regnn_hip import build as B  # noqa: E402


def main():
    name, extra = sys.argv[1], sys.argv[2:]
    od = os.path.join(ROOT, os.environ.get("AB_DIR", "ab"), f"obj_{name}")
    os.makedirs(od, exist_ok=True)

    def comp(src):
        obj = os.path.join(od, os.path.basename(src)[:-4] + ".o")
        r = subprocess.run([B.HIPCC, *B.FLAGS, *extra, "-c", src, "-o", obj],
                           capture_output=True, text=True)
        if r.returncode:
            raise RuntimeError(r.stderr)
        return obj
    with cf.ThreadPoolExecutor(8) as ex:
        objs = list(ex.map(comp, B._sources()))
    out = os.path.join(ROOT, os.environ.get("AB_DIR", "ab"), f"libregnn_{name}.so")
    r = subprocess.run([B.HIPCC, "-shared", "-fPIC", f"--offload-arch={B.ARCH}", *objs, "-o", out],
                       capture_output=True, text=True)
    if r.returncode:
        raise RuntimeError(r.stderr)
    print(out)


if __name__ == "__main__":
    main()
