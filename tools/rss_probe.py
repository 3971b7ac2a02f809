"""Peak host RSS of salz CLI runs (diagnostic): python tools/rss_probe.py <size> <level> ..."""
import os
import resource
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from tests.helpers import gen  # noqa: E402

cli = os.path.join(ROOT, "salz_amd", "salz")
args = sys.argv[1:]
for size, level in zip(args[0::2], args[1::2]):
    f = f"/tmp/rss_{size}.txt"
    gen("text", int(size), 3).tofile(f)
    probe = ("import resource, subprocess, sys; r = subprocess.run(sys.argv[1:]); "
             "print(r.returncode, resource.getrusage(resource.RUSAGE_CHILDREN).ru_maxrss)")
    out = subprocess.run([sys.executable, "-c", probe, cli, f"-{level}", "-k", "-q", "-f", f],
                         capture_output=True, text=True).stdout.split()
    print(f"size {size} level {level}: rc {out[-2]} peak RSS {int(out[-1]) / 1024:.0f} MiB", flush=True)
    os.unlink(f)
    if os.path.exists(f + ".salz"):
        os.unlink(f + ".salz")
