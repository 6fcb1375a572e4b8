"""Build time of the terrain's fine-window copy (pcp_fine.hip, sorted with rocPRIM directly):
the index_build profile slot around the query that triggers it (PCP_TERRAIN_BLOCKS=2: the first
query) on the C2 terrain, minus the same query's slot with the copy already built.  Prints one
JSON line (profiles/r03_fine_build_time.json)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

os.environ["PCP_TERRAIN_BLOCKS"] = "2"
from pointcloud_processor_amd import _abi, synth  # noqa: E402

sc = synth.terrain_scene()
poses = np.array([[8.0, -3.0, 1.1, -0.5, 2.6]])
fan = _abi.fan_params(n_az=64, n_el=4)
res = []
for rep in range(6):
    ctx = _abi.Context(0)
    ctx.set_terrain(sc.terrain, point_step=32)
    ctx.profile(True)
    ctx.profile_reset()
    ctx.raycast_fan(poses, fan)          # builds the fine copy, then marches
    ms, n = ctx.profile_get("index_build")
    info = ctx.terrain_info()
    ctx.close()
    res.append(ms)
print(json.dumps({"what": "fine-window copy build (k_zkeys, rocprim radix sort x2, window "
                          "count/emit/bounds/place, records, pack) of the 1,001,740-pt C2 terrain",
                  "ms_runs": res, "ms_median": float(np.median(res[1:])),
                  "scan_layout": info["scan_layout"], "fine_tile": info["fine_tile"]}))
