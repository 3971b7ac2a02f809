"""Peak host RSS of the HIP runtime itself (diagnostic): after device discovery, after one
encoder context, after one 1 MiB encode."""
import os
import resource
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import salz_amd  # noqa: E402
from tests.helpers import gen  # noqa: E402


def rss():
    return resource.getrusage(resource.RUSAGE_SELF).ru_maxrss / 1024


print(f"python + libsalz loaded: {rss():.0f} MiB")
salz_amd.device_count()
print(f"after hipGetDeviceCount: {rss():.0f} MiB")
c = salz_amd.Context(0, 1 << 20)
print(f"after one context (1 MiB workspace): {rss():.0f} MiB")
c.encode(gen("text", 1 << 20, 1))
print(f"after one 1 MiB encode: {rss():.0f} MiB")
