"""Run an unmodified reference driver (e.g. RE-GNN's run_regnn.py) on the MI355X build.

    python -m regnn_hip.run /path/to/RE-GNN/run_regnn.py --dataset DBLP --model regcn ...

Python would put the script's own directory first on sys.path, so the checkout's ``layer/``
package would shadow the drop-in one. This launcher orders the path as [this build (layer, dgl),
the script's directory (model, utils, ...), ...] and executes the script as ``__main__``.
"""
import os
import runpy
import sys

PKG_DIR = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main(argv=None):
    argv = list(sys.argv[1:] if argv is None else argv)
    if not argv:
        raise SystemExit(__doc__)
    script = os.path.abspath(argv[0])
    for p in (os.path.dirname(script), PKG_DIR):
        if p in sys.path:
            sys.path.remove(p)
        sys.path.insert(0, p)
    sys.path.remove(PKG_DIR)
    sys.path.insert(0, PKG_DIR)
    sys.argv = [script] + argv[1:]
    runpy.run_path(script, run_name="__main__")


if __name__ == "__main__":
    main()
