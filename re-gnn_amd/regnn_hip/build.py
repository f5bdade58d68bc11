"""Build libregnn_hip.so (the C-ABI of include/regnn_hip.h) in-tree for gfx950 with hipcc.

    python -m regnn_hip.build          (from re-gnn_amd/)   or   __graft_entry__.build()

Compiles every csrc/*.hip to an object (in parallel), links one shared library next to this file.
Freshness is decided by content, not mtime: the library is rebuilt unless its sidecar
``libregnn_hip.so.hash`` holds the SHA-256 of every source, header and build flag AND the library
reports the ABI version include/regnn_hip.h declares.
"""
import concurrent.futures as cf
import ctypes
import glob
import hashlib
import os
import re
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.dirname(HERE)
CSRC = os.path.join(PKG, "csrc")
INCLUDE = os.path.join(os.path.dirname(PKG), "include")
LIB = os.path.join(HERE, "libregnn_hip.so")
HASH = LIB + ".hash"
OBJDIR = os.path.join(PKG, "build")
ARCH = os.environ.get("REGNN_OFFLOAD_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
FLAGS = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-I", INCLUDE,
         "-Wno-unused-result"]


def _flags_key():
    """the compiler flags with the include path made repo-relative: a hash of them is the same
    in every checkout (here and on the GPU box)."""
    root = os.path.dirname(PKG)
    return " ".join(os.path.relpath(f, root) if os.path.isabs(f) else f for f in FLAGS)


def _sources():
    return sorted(glob.glob(os.path.join(CSRC, "*.hip")))


def _deps():
    return sorted(_sources() + glob.glob(os.path.join(CSRC, "*.h")) +
                  glob.glob(os.path.join(INCLUDE, "*.h")))


def source_hash():
    """SHA-256 over the kernel sources, headers and compiler flags (also keys the committed
    rocprofv3 counter summaries in profiles/ to the code they were measured on)."""
    h = hashlib.sha256()
    for p in _deps():
        h.update(os.path.relpath(p, os.path.dirname(PKG)).encode())
        with open(p, "rb") as f:
            h.update(f.read())
    h.update(_flags_key().encode())
    return h.hexdigest()


# the kernels the committed rocprofv3 counter summaries measure (bench.py pmc_traffic): their
# sources alone key the summaries, so a change elsewhere (e.g. the NS engine) keeps them valid
PMC_SOURCES = ("re_spmm.hip", "re_dense.hip", "regnn_common.h")
# the fused NS model step's kernels (profiles/pmc_ns_fp32.json)
NS_PMC_SOURCES = ("re_nsm.hip", "re_nsm2.hip", "re_nsm_common.h", "regnn_common.h")
NS_SUMS_SOURCES = ("re_ns.hip", "regnn_common.h")             # the sampler's sums launch


def kernel_hash(names=PMC_SOURCES):
    """SHA-256 over the named csrc/ files and the compiler flags."""
    h = hashlib.sha256()
    for name in names:
        with open(os.path.join(CSRC, name), "rb") as f:
            h.update(name.encode())
            h.update(f.read())
    h.update(_flags_key().encode())
    return h.hexdigest()


def header_abi():
    with open(os.path.join(INCLUDE, "regnn_hip.h")) as f:
        m = re.search(r"ABI version \(.*?currently (\d+)\)", f.read(), re.S)
    return int(m.group(1)) if m else None


def _lib_abi():
    try:
        return int(ctypes.CDLL(LIB).regnn_abi_version())
    except OSError:
        return None


def up_to_date():
    if not (os.path.exists(LIB) and os.path.exists(HASH)):
        return False
    with open(HASH) as f:
        if f.read().strip() != source_hash():
            return False
    return _lib_abi() == header_abi()


def _compile(src):
    obj = os.path.join(OBJDIR, os.path.basename(src)[:-4] + ".o")
    cmd = [HIPCC, *FLAGS, "-c", src, "-o", obj]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed for {src}:\n{r.stdout}\n{r.stderr}")
    return obj


def build(force=False, verbose=True):
    if not force and up_to_date():
        return LIB
    digest = source_hash()
    os.makedirs(OBJDIR, exist_ok=True)
    srcs = _sources()
    with cf.ThreadPoolExecutor(max_workers=min(8, len(srcs))) as ex:
        objs = list(ex.map(_compile, srcs))
    tmp = LIB + ".tmp"
    cmd = [HIPCC, "-shared", "-fPIC", f"--offload-arch={ARCH}", *objs, "-o", tmp]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"link failed:\n{r.stdout}\n{r.stderr}")
    os.replace(tmp, LIB)
    with open(HASH, "w") as f:
        f.write(digest + "\n")
    if _lib_abi() != header_abi():
        raise RuntimeError(f"built library reports ABI {_lib_abi()}, header declares "
                           f"{header_abi()}")
    if verbose:
        print(f"[regnn_hip] built {LIB} ({len(srcs)} sources, {ARCH})", file=sys.stderr)
    return LIB


if __name__ == "__main__":
    build(force="--force" in sys.argv)
