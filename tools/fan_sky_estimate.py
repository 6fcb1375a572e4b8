# The fan A/B idea "a wave-uniform probe for a ring's samples that all lie above the terrain"
# (VERDICT r02 item 8), bounded on the CPU before building it: the fraction of in-box fan samples
# (an upper bound of the probes) that a wave-uniform test could skip -- sample z - (r + m) above
# the max terrain z over the xy bbox of the wave's 64 samples (inflated by r + m), on 0.12 m
# columns.  16 of the 256 C2 poses, every 4th ring.  Output: profiles/r03_fan_ab_sky_estimate.log
import sys, math, numpy as np
sys.path.insert(0, '.'); sys.path.insert(0, 'oracle')
from pointcloud_processor_amd import synth
sc = synth.terrain_scene()
T = sc.terrain[:, :3].astype(np.float64)
R = 0.056 + 0.001
# coarse max-height grid at 0.12 m
c = 0.12
ox, oy = T[:, 0].min() - 1, T[:, 1].min() - 1
ix = ((T[:, 0] - ox) / c).astype(int); iy = ((T[:, 1] - oy) / c).astype(int)
nx, ny = ix.max() + 2, iy.max() + 2
H = np.full((ny, nx), -np.inf)
np.maximum.at(H, (iy, ix), T[:, 2])
bb = T.min(0) - R, T.max(0) + R
import bench
from pointcloud_processor_amd import _abi
# poses: reuse the candidate lattice via oracle generator
import pyoracle
Tc = pyoracle.Cloud(sc.terrain)
params = pyoracle.vl_params(num_candidates=348)
poses = pyoracle.generate_candidates(Tc, bench._grid_bbox(sc.area), params, sc.zx120_pose5)[:256:16]
n_az, n_el = 1024, 256
el = np.deg2rad(-85 + 170 * (np.arange(n_el) + 0.5) / n_el)
az = 2 * np.pi * np.arange(n_az) / n_az
steps = [0.5]
while steps[-1] + 0.3 < 15 - 0.08: steps.append(steps[-1] + 0.3)
S = np.array(steps)
tot = skip = 0
for p in poses:
    px, py, pz, pitch, yaw = p
    for j in range(0, n_el, 4):          # every 4th ring
        ce, se = math.cos(el[j]), math.sin(el[j])
        for w in range(0, n_az, 64):
            a = az[w:w + 64] + yaw
            ux, uy = ce * np.cos(a), ce * np.sin(a)
            # samples inside the bbox per lane
            qx = px + np.outer(ux, S); qy = py + np.outer(uy, S); qz = pz + se * S
            inb = (qx > bb[0][0]) & (qx < bb[1][0]) & (qy > bb[0][1]) & (qy < bb[1][1]) & (qz[None, :] > bb[0][2]) & (qz[None, :] < bb[1][2])
            cnt = inb.sum(0)
            ks = np.nonzero(cnt)[0]
            for k in ks:
                m = inb[:, k]
                x0, x1 = qx[m, k].min() - R, qx[m, k].max() + R
                y0, y1 = qy[m, k].min() - R, qy[m, k].max() + R
                gx0, gx1 = max(int((x0 - ox) / c), 0), min(int((x1 - ox) / c), nx - 1)
                gy0, gy1 = max(int((y0 - oy) / c), 0), min(int((y1 - oy) / c), ny - 1)
                h = H[gy0:gy1 + 1, gx0:gx1 + 1].max() if gx1 >= gx0 and gy1 >= gy0 else -np.inf
                tot += cnt[k]
                if qz[k] - R > h: skip += cnt[k]
print("in-box samples (upper bound of probes):", tot, "skippable:", skip, f"{skip / max(tot, 1):.3f}")
