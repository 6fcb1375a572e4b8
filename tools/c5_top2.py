"""The full-chain C5 replay (pcp_nodes_cli replay, chain mode) with its frame dumps, each dumped
frame re-run through the oracle chain ON ITS OWN (its own filtered clouds, carve, normals,
cells, candidates -- never a GPU output), and per frame: the best index of both, the largest
relative total difference, and the top-2 relative gap of the oracle's totals (how far the
argmax is from flipping).  -> profiles/r04_c5_top2_gaps.json (run on the GPU box:
python tools/c5_top2.py FRAMES OUT)."""
import json
import math
import subprocess
import sys
import tempfile
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "oracle"))


def main():
    frames = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    out = Path(sys.argv[2]) if len(sys.argv) > 2 else ROOT / "profiles" / "r04_c5_top2_gaps.json"
    import pyoracle as oracle
    from pointcloud_processor_amd import synth

    sc = synth.terrain_scene()
    cells = synth.excavation_cells(sc.area)
    d = Path(tempfile.mkdtemp(prefix="pcp_top2_"))
    np.ascontiguousarray(sc.terrain).tofile(d / "t.f32")
    np.ascontiguousarray(cells.xyz).tofile(d / "c.f64")
    np.ascontiguousarray(cells.normals).tofile(d / "n.f32")
    bb = ",".join(repr(float(v)) for v in cells.grid_bbox)
    cli = ROOT / "pointcloud_processor_amd" / "_lib" / "pcp_nodes_cli"
    r = subprocess.run([str(cli), "replay", str(d / "t.f32"), str(sc.terrain.shape[0]),
                        str(d / "c.f64"), str(d / "n.f32"), str(cells.xyz.shape[0]), bb,
                        str(frames), "60032", "1", str(d)], capture_output=True, text=True,
                       timeout=600, check=True)
    res = json.loads(r.stdout.strip().splitlines()[-1])
    box = np.array([0.0, 15.0, -10.0, 10.0, -1.5, 10.0])
    rt = ((8.0, -3.0, 2.0), (0.0, 0.0, 0.2588190451025208, 0.9659258262890683))
    zt = ((0.55, 0.4, 3.5), (0.0, 0.21633, 0.0, 0.97632))
    zx = np.array([0.4, 0.5, 3.5, -math.pi / 6, 0.0])
    rows = []
    for fr in res["dumped"]:
        pre = f"f{fr['frame']}_"
        ld = lambda name, dt, cols: np.fromfile(d / (pre + name), dt).reshape(-1, cols)
        filt = []
        for tag in ("rscan", "zscan"):
            scan = ld(tag + ".f32", np.float32, 4)
            vox, _, _, _ = oracle.voxel_grid(scan[oracle.crop_box(scan, box)], 0.2)
            filt.append(vox)
        ref = np.concatenate([oracle.transform_rgb(filt[0], rt[0], rt[1], (255, 0, 0)),
                              oracle.transform_rgb(filt[1], zt[0], zt[1], (0, 0, 255))])
        keep, surf, area, _ = oracle.excavate(ref, (0.0, 0.0, 0.0), (0.0, 0.0, 0.0, 1.0))
        terr = np.concatenate([ref[keep][:, [0, 1, 2, 4]], surf])
        r_n = oracle.area_normals(area, 1.5)
        xyz, cn, gbb, _ = oracle.excavation_grid(area, 0.1, 10, r_n)
        T = oracle.Cloud(terr)
        poses = oracle.generate_candidates(T, gbb, oracle.vl_params(), zx)
        aux = np.zeros((filt[1].shape[0], 4), np.float32)
        aux[:, :3] = filt[1]
        tot, _, rep = oracle.score_poses(T, oracle.Cloud(aux), xyz, cn, poses, zx,
                                         oracle.vl_params(), np.zeros(xyz.shape[0], np.uint8))
        got = np.fromfile(d / (pre + "tot.f64"), np.float64)
        gcn = ld("cnrm.f32", np.float32, 3)
        srt = np.sort(tot)[::-1]
        rows.append({
            "frame": fr["frame"], "candidates": int(tot.size), "cells": int(xyz.shape[0]),
            "best_idx_gpu": int(fr["best_idx"]), "best_idx_oracle": int(rep.best_idx),
            "cell_normals_bit_identical": bool(gcn.shape == cn.shape and
                                               np.array_equal(gcn.view(np.uint32), cn.view(np.uint32))),
            "max_rel_total_diff": float(np.max(np.abs(got - tot) / np.maximum(np.abs(tot), 1e-300)))
            if got.shape == tot.shape and tot.size else None,
            "top2_rel_gap": float((srt[0] - srt[1]) / abs(srt[0])) if srt.size >= 2 and srt[0] else None,
        })
        print(rows[-1], flush=True)
    out.write_text(json.dumps({"source": "tools/c5_top2.py", "frames_replayed": frames,
                               "rows": rows}, indent=2) + "\n")


if __name__ == "__main__":
    main()
