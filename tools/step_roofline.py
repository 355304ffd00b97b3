"""Step-kernel HBM roofline over batch sizes (bench.step_kernel_point per row).

Rows: the headline 4096 x 12x12 (latency-bound), 65,536 x 20x20 (working set
inside the 256 MB Infinity Cache) and 262,144 x 20x20 (HBM-resident), pure
step and with the replay store fused. One JSON line per row.
"""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
import bench  # noqa: E402
import snake_amd as snk  # noqa: E402

snk.load()
for n, bs, store in [(4096, 12, True), (65536, 20, False), (65536, 20, True), (262144, 20, False),
                     (262144, 20, True), (262144, 12, True)]:
    print(json.dumps(bench.step_kernel_point(snk, n, bs, 2, store)), flush=True)
