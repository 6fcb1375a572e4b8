/*
 * pcp_oracle_mt.c -- the C3 frame (crop + VoxelGrid + transform + colour + concat) on all host
 * threads with OpenMP.  TEST INFRASTRUCTURE ONLY: the multi-threaded CPU baseline of
 * bench.py's c3 workload ("1 thread + OpenMP").  The reference path is
 * single-threaded (pointcloud_filter.cpp:64-139, pointcloud_merger.cpp:354-394); this file
 * parallelises the same arithmetic and produces the same bytes as the sequential
 * orc_crop_box -> orc_voxel_grid -> orc_transform_rgb composition (tests/test_oracle.py):
 *  - crop: per-thread chunks counted, then written at their prefix (input order kept);
 *  - VoxelGrid: keys as applyFilter computes them, a stable LSD radix sort of (key, input
 *    index) (= the (idx, cloud_index) order orc_voxel_grid's qsort fixes), voxel runs found
 *    in parallel, each centroid summed in input order by one thread;
 *  - transform: the Eigen float expression per point.
 */
#include "pcp_oracle.h"

#include <float.h>
#include <math.h>
#include <stdlib.h>
#include <string.h>
#include <omp.h>

typedef struct { uint32_t key; uint32_t idx; } mt_pair;

/* stable LSD radix sort of pairs by key (11-bit digits), per-thread histograms */
static void mt_radix_sort(mt_pair *a, mt_pair *tmp, int64_t m, int T)
{
    enum { BITS = 11, BINS = 1 << BITS };
    uint32_t maxk = 0;
#pragma omp parallel for reduction(max : maxk) num_threads(T)
    for (int64_t i = 0; i < m; ++i)
        if (a[i].key > maxk) maxk = a[i].key;
    int passes = 0;
    while (passes * BITS < 32 && (maxk >> (passes * BITS)) != 0) ++passes;
    int64_t *hist = (int64_t *)calloc((size_t)T * BINS, sizeof(int64_t));
    for (int p = 0; p < passes; ++p) {
        const int sh = p * BITS;
        memset(hist, 0, (size_t)T * BINS * sizeof(int64_t));
#pragma omp parallel num_threads(T)
        {
            const int t = omp_get_thread_num(), nt = omp_get_num_threads();
            const int64_t lo = m * t / nt, hi = m * (t + 1) / nt;
            int64_t *h = hist + (size_t)t * BINS;
            for (int64_t i = lo; i < hi; ++i) ++h[(a[i].key >> sh) & (BINS - 1)];
#pragma omp barrier
#pragma omp single
            {   /* digit-major, thread-minor offsets: stable */
                int64_t s = 0;
                for (int d = 0; d < BINS; ++d)
                    for (int u = 0; u < nt; ++u) {
                        const int64_t c = hist[(size_t)u * BINS + d];
                        hist[(size_t)u * BINS + d] = s;
                        s += c;
                    }
            }
            for (int64_t i = lo; i < hi; ++i) tmp[h[(a[i].key >> sh) & (BINS - 1)]++] = a[i];
        }
        mt_pair *x = a;
        a = tmp;
        tmp = x;
    }
    if (passes & 1) memcpy(tmp, a, (size_t)m * sizeof(mt_pair));   /* result back in the caller's a */
    free(hist);
}

/* one cloud: crop (box) -> VoxelGrid (leaf) -> centroids (xyz, 3 floats each); returns the
 * count, *passthrough as orc_voxel_grid */
static int64_t mt_crop_voxel(const float *pts, int64_t n, int64_t stride, const double box[6],
                             float leaf, int T, float **out_xyz)
{
    /* cropFrontArea (pointcloud_filter.cpp:106-116) */
    int64_t *cnt = (int64_t *)calloc((size_t)T + 1, sizeof(int64_t));
    uint32_t *kept = (uint32_t *)malloc((size_t)(n ? n : 1) * sizeof(uint32_t));
#pragma omp parallel num_threads(T)
    {
        const int t = omp_get_thread_num(), nt = omp_get_num_threads();
        const int64_t lo = n * t / nt, hi = n * (t + 1) / nt;
        int64_t c = 0;
        for (int64_t i = lo; i < hi; ++i) {
            const float *p = pts + i * stride;
            c += (double)p[0] > box[0] && (double)p[0] < box[1] && (double)p[1] > box[2] &&
                 (double)p[1] < box[3] && (double)p[2] > box[4] && (double)p[2] < box[5];
        }
        cnt[t + 1] = c;
#pragma omp barrier
#pragma omp single
        for (int u = 0; u < nt; ++u) cnt[u + 1] += cnt[u];
        int64_t w = cnt[t];
        for (int64_t i = lo; i < hi; ++i) {
            const float *p = pts + i * stride;
            if ((double)p[0] > box[0] && (double)p[0] < box[1] && (double)p[1] > box[2] &&
                (double)p[1] < box[3] && (double)p[2] > box[4] && (double)p[2] < box[5])
                kept[w++] = (uint32_t)i;
        }
    }
    int64_t m = 0;
    for (int u = 0; u < T; ++u) m = cnt[u + 1] > m ? cnt[u + 1] : m;
    free(cnt);
    float *out = (float *)malloc((size_t)(m ? m : 1) * 3 * sizeof(float));
    *out_xyz = out;
    if (m == 0) {
        free(kept);
        return 0;
    }
    /* VoxelGrid<PointXYZ>::applyFilter: bbox of the (finite) cropped points */
    const float inv = 1.0f / leaf;
    float mn0 = FLT_MAX, mn1 = FLT_MAX, mn2 = FLT_MAX, mx0 = -FLT_MAX, mx1 = -FLT_MAX, mx2 = -FLT_MAX;
#pragma omp parallel for num_threads(T) reduction(min : mn0, mn1, mn2) reduction(max : mx0, mx1, mx2)
    for (int64_t j = 0; j < m; ++j) {
        const float *p = pts + (int64_t)kept[j] * stride;
        mn0 = fminf(mn0, p[0]); mn1 = fminf(mn1, p[1]); mn2 = fminf(mn2, p[2]);
        mx0 = fmaxf(mx0, p[0]); mx1 = fmaxf(mx1, p[1]); mx2 = fmaxf(mx2, p[2]);
    }
    const int64_t dxl = (int64_t)((mx0 - mn0) * inv) + 1, dyl = (int64_t)((mx1 - mn1) * inv) + 1,
                  dzl = (int64_t)((mx2 - mn2) * inv) + 1;
    if (dxl * dyl * dzl > (int64_t)INT32_MAX) {   /* PCL's overflow guard: passthrough */
#pragma omp parallel for num_threads(T)
        for (int64_t j = 0; j < m; ++j)
            for (int a = 0; a < 3; ++a) out[3 * j + a] = pts[(int64_t)kept[j] * stride + a];
        free(kept);
        return m;
    }
    const int min_b0 = (int)floorf(mn0 * inv), min_b1 = (int)floorf(mn1 * inv),
              min_b2 = (int)floorf(mn2 * inv);
    const int mul1 = (int)floorf(mx0 * inv) - min_b0 + 1;
    const int mul2 = mul1 * ((int)floorf(mx1 * inv) - min_b1 + 1);
    mt_pair *iv = (mt_pair *)malloc((size_t)m * sizeof(mt_pair));
    mt_pair *tmp = (mt_pair *)malloc((size_t)m * sizeof(mt_pair));
#pragma omp parallel for num_threads(T)
    for (int64_t j = 0; j < m; ++j) {
        const float *p = pts + (int64_t)kept[j] * stride;
        const int i0 = (int)(floorf(p[0] * inv) - (float)min_b0);
        const int i1 = (int)(floorf(p[1] * inv) - (float)min_b1);
        const int i2 = (int)(floorf(p[2] * inv) - (float)min_b2);
        iv[j].key = (uint32_t)(i0 + i1 * mul1 + i2 * mul2);
        iv[j].idx = kept[j];
    }
    free(kept);
    mt_radix_sort(iv, tmp, m, T);
    /* voxel runs: heads counted per chunk, then each voxel summed in input order */
    int64_t *hc = (int64_t *)calloc((size_t)T + 1, sizeof(int64_t));
    int64_t nv = 0;
#pragma omp parallel num_threads(T)
    {
        const int t = omp_get_thread_num(), nt = omp_get_num_threads();
        const int64_t lo = m * t / nt, hi = m * (t + 1) / nt;
        int64_t c = 0;
        for (int64_t i = lo; i < hi; ++i) c += i == 0 || iv[i].key != iv[i - 1].key;
        hc[t + 1] = c;
#pragma omp barrier
#pragma omp single
        {
            for (int u = 0; u < nt; ++u) hc[u + 1] += hc[u];
            nv = hc[nt];
        }
        int64_t v = hc[t];
        for (int64_t i = lo; i < hi; ++i) {
            if (!(i == 0 || iv[i].key != iv[i - 1].key)) continue;
            int64_t e = i + 1;
            while (e < m && iv[e].key == iv[i].key) ++e;
            float sx = 0.f, sy = 0.f, sz = 0.f;   /* CentroidPoint: float sums in order */
            for (int64_t l = i; l < e; ++l) {
                const float *p = pts + (int64_t)iv[l].idx * stride;
                sx += p[0]; sy += p[1]; sz += p[2];
            }
            const float c = (float)(e - i);
            out[3 * v] = sx / c;
            out[3 * v + 1] = sy / c;
            out[3 * v + 2] = sz / c;
            ++v;
        }
    }
    free(hc);
    free(iv);
    free(tmp);
    return nv;
}

int64_t orc_filter_frame_mt(int k, const float *const *pts, const int64_t *n,
                            const int64_t *stride, const double *boxes, float leaf,
                            const double *t3q4, const uint8_t *rgb, float *out8, int64_t cap,
                            int64_t *n_per, int threads)
{
    const int T = threads > 0 ? threads : 1;
    int64_t base = 0;
    for (int c = 0; c < k; ++c) {
        float *xyz = NULL;
        const int64_t nv = leaf > 0.0f
                               ? mt_crop_voxel(pts[c], n[c], stride[c], boxes + 6 * c, leaf, T, &xyz)
                               : -1;
        if (nv < 0) return -1;   /* crop-only frames are not a C3 workload */
        if (base + nv > cap) {
            free(xyz);
            return -1;
        }
        /* processRobotCloud's doTransform + colour (pointcloud_merger.cpp:354-394) */
        const double *tq = t3q4 + 7 * c;
        const int64_t chunk = 1 << 14;
#pragma omp parallel for num_threads(T) schedule(static)
        for (int64_t s = 0; s < nv; s += chunk)
            orc_transform_rgb(xyz + 3 * s, (nv - s) < chunk ? nv - s : chunk, 3, tq, tq + 3,
                              rgb[3 * c], rgb[3 * c + 1], rgb[3 * c + 2], out8 + 8 * (base + s));
        free(xyz);
        if (n_per) n_per[c] = nv;
        base += nv;
    }
    return base;
}
