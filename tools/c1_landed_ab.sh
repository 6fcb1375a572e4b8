# C1 A/B: the carve's messages copied by pcp_excavate_area_async (PCP_C1_LANDED=0) or read from
# its landing after the zx120 index is enqueued (1, default); alternating processes
for r in 1 2 3; do for v in 0 1; do PCP_C1_LANDED=$v timeout -k 10 200 python bench.py --mode c1 --steps 30 --warmup 5 > gpurun_out/c1l_$v.json 2>gpurun_out/c1l_$v.err || exit 1; python3 -c "
import json; d=[json.loads(l) for l in open('gpurun_out/c1l_$v.json') if l.startswith('{')][-1]; c=d.get('c1', d); print('r$r landed=$v', 'p50 %.4f p99 %.4f' % (c['value'], c['p99_ms']), 'matches', c.get('matches_oracle'), c.get('best_idx_matches_oracle'), c.get('totals_bar'))"; done; done
