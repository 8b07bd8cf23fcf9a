"""Per-round kernel time of a simulator run from a rocprofv3 results database: the run whose
k_sim_init is the idx-th (0 = C4, 1 = C5 in bench.py's order), rounds split at k_round_begin.

    python tools/sim_rounds_db.py gpurun_out/x/run_results.db [idx]"""
import sqlite3
import sys

db = sys.argv[1]
idx = int(sys.argv[2]) if len(sys.argv) > 2 else 1
c = sqlite3.connect(db)
rows = list(c.execute("select name, start, end, grid_x, workgroup_x from kernels order by start"))
inits = [i for i, r in enumerate(rows) if 'k_sim_init' in r[0]]
seg_all = rows[inits[idx]: inits[idx + 1] if idx + 1 < len(inits) else len(rows)]
rb = [i for i, r in enumerate(seg_all) if 'k_round_begin' in r[0]]
names = ['k_ck_lanes', 'k_ck_pair', 'k_ck_pc<7, 4>', 'k_ck_pc<3, 2>', 'k_phase_b', 'k_phase_c', 'k_phase_e', 'k_phase_a',
         'k_phase_d1', 'k_phase_d2', 'k_twin', 'k_out_fill', 'k_conv_local']
print('round  wall ', ' '.join('%7s' % n.replace('k_', '').replace('phase_', 'p')[:7] for n in names), ' busy')
tot = {n: 0.0 for n in names}
W = B = 0.0
for j in range(len(rb)):
    seg = seg_all[rb[j]: rb[j + 1] if j + 1 < len(rb) else len(seg_all)]
    wall = (seg[-1][2] - seg[0][1]) / 1e6
    busy = sum((r[2] - r[1]) / 1e6 for r in seg)
    W += wall
    B += busy
    t = {n: sum((r[2] - r[1]) / 1e6 for r in seg if n in r[0]) for n in names}
    for n in names:
        tot[n] += t[n]
    print('%3d %7.1f ' % (j, wall), ' '.join('%7.1f' % t[n] for n in names), '%6.1f' % busy)
print('total wall %.1f busy %.1f' % (W, B))
print(' '.join('%s=%.0f' % (n, v) for n, v in tot.items()))
