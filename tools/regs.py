"""Register / spill report of the gfx950 kernels in one csrc file (hipcc --save-temps metadata).

    python tools/regs.py re_dense [name-substring ...]
"""
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    src = os.path.join(ROOT, "re-gnn_amd", "csrc", sys.argv[1] + ".hip")
    pats = sys.argv[2:]
    with tempfile.TemporaryDirectory() as d:
        subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950",
                        "-I", os.path.join(ROOT, "include"), "--save-temps", "-c", src,
                        "-o", os.path.join(d, "k.o")], cwd=d, check=True,
                       stderr=subprocess.DEVNULL)
        asm = [f for f in os.listdir(d) if f.endswith("gfx950.s")][0]
        s = open(os.path.join(d, asm)).read()
    meta = s[s.index("amdhsa.kernels:"):]
    for b in re.split(r"\n  - ", meta):
        nm = re.search(r"\.name:\s+(\S+)", b)
        if not nm or (pats and not any(p in nm.group(1) for p in pats)):
            continue

        def g(k):
            m = re.search(r"\." + k + r":\s+(\d+)", b)
            return m.group(1) if m else None
        print(f"{nm.group(1)[:70]:72s} vgpr {g('vgpr_count')} agpr {g('agpr_count')} "
              f"sgpr-spill {g('sgpr_spill_count')} vgpr-spill {g('vgpr_spill_count')}")


if __name__ == "__main__":
    main()
