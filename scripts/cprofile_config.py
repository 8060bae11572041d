"""cProfile one bench config (host-side hot spots of an API bench on the GPU box):
python scripts/cprofile_config.py <out.txt> <bench_configs args...>"""
import cProfile
import io
import os
import pstats
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from mxstream.models import bench_configs  # noqa: E402

out = sys.argv[1]
prof = cProfile.Profile()
prof.enable()
bench_configs.main(sys.argv[2:])
prof.disable()
s = io.StringIO()
st = pstats.Stats(prof, stream=s)
st.sort_stats("tottime").print_stats(40)
st.sort_stats("cumulative").print_stats(40)
st.print_callers("torch.empty|absorb|export|query")
with open(out, "w") as f:
    f.write(s.getvalue())
