"""bench.py with engine knobs set first (diagnostics): python3 tools/bench_knobs.py key=value
... -- <bench.py args>"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
i = sys.argv.index("--") if "--" in sys.argv else len(sys.argv)
knobs = [a.split("=") for a in sys.argv[1:i]]
sys.argv = [os.path.join(REPO, "bench.py")] + sys.argv[i + 1:]
import bench  # noqa: E402

_load = bench.load_pkg


def load_pkg():
    pg = _load()
    for k, v in knobs:
        pg.lib.pgcn_debug_set(k.encode(), int(v))
    return pg


bench.load_pkg = load_pkg
bench.main()
