"""Host-side hot spots of the serving loop: run bench.py under cProfile and print the functions
with the largest own time (tottime) and cumulative time, excluding the GPU wait."""
import cProfile
import os
import pstats
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
out = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/bench.prof"
sys.argv = ["bench.py"] + sys.argv[2:]
import runpy  # noqa: E402

cProfile.run("runpy.run_path(os.path.join(ROOT, 'bench.py'), run_name='__main__')", out)
st = pstats.Stats(out)
st.sort_stats("tottime").print_stats(35)
st.sort_stats("cumulative").print_stats(45)
