"""Build libregnn_hip.so from the kernel sources of a git revision (A/B against the working tree:
load it on the GPU box through REGNN_LIB). usage: python tools/build_rev.py REV NAME [-DFLAG ...]
-> ab/libregnn_NAME.so. The revision's include/regnn_hip.h must carry the same ABI version as the
Python side that loads it."""
import concurrent.futures as cf
import os
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "re-gnn_amd"))
from regnn_hip import build as B  # noqa: E402


def main():
    rev, name, extra = sys.argv[1], sys.argv[2], sys.argv[3:]
    files = subprocess.run(["git", "ls-tree", "-r", "--name-only", rev, "re-gnn_amd/csrc",
                            "include"], cwd=ROOT, capture_output=True, text=True,
                           check=True).stdout.split()
    with tempfile.TemporaryDirectory() as d:
        for f in files:
            os.makedirs(os.path.join(d, os.path.dirname(f)), exist_ok=True)
            with open(os.path.join(d, f), "wb") as o:
                o.write(subprocess.run(["git", "show", f"{rev}:{f}"], cwd=ROOT,
                                       capture_output=True, check=True).stdout)
        srcs = [os.path.join(d, f) for f in files if f.endswith(".hip")]
        flags = [x if x != B.INCLUDE else os.path.join(d, "include") for x in B.FLAGS]

        def comp(src):
            obj = src[:-4] + ".o"
            r = subprocess.run([B.HIPCC, *flags, *extra, "-c", src, "-o", obj],
                               capture_output=True, text=True)
            if r.returncode:
                raise RuntimeError(r.stderr)
            return obj
        with cf.ThreadPoolExecutor(8) as ex:
            objs = list(ex.map(comp, srcs))
        os.makedirs(os.path.join(ROOT, "ab"), exist_ok=True)
        out = os.path.join(ROOT, "ab", f"libregnn_{name}.so")
        subprocess.run([B.HIPCC, "-shared", "-fPIC", f"--offload-arch={B.ARCH}", *objs, "-o", out],
                       check=True)
    print(out)


if __name__ == "__main__":
    main()
