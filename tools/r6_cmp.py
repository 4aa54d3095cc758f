"""Round-6 summary of bench detail files (tuning); sections a run skipped
(--anchor-log-n 0, --no-pcie, --no-msm, --no-cpu-baseline) are left out."""
import json
import sys

for f in sys.argv[1:]:
    d = json.load(open(f))
    print(f)
    pc = (d.get('pcie_inclusive') or {}).get('over_resident_ms')
    line = [' prove', d['ms_per_step'], 'bit_exact', d.get('bit_exact_vs_oracle'), 'pcie+', pc]
    if d.get('ntt'):
        line += ['ntt', d['ntt']['ms_per_ntt']]
    m = d.get('msm_g1')
    if m:
        line += ['msm_g1', m['ms_per_msm'], m['plain']['ms_per_msm'], m['bits64']['ms_per_msm']]
    r = d['roofline']
    line += ['roof', r['frac'], r['avg_launch_ms'], r['valu']['frac']]
    print(*line)
    a = d.get('strong_scaling_anchor')
    if a:
        print(' anchor', a['ms_per_step'], 'msm_only', a['msm_only']['ms_per_step'], a['bit_exact_vs_oracle'], 'c16',
              a['same_plan_c16']['msm_only']['ms_per_step'], a['same_plan_c16']['ms_per_step'])
        s = a.get('shard8_msm_only')
        if s:
            print(' shard', s['ms_per_step'], s['phases_ms_slowest'], s['msm_scaling_projected'],
                  s['folded_proof_bit_exact_vs_anchor'], s.get('per_shard_ms'))
    ss = d.get('serial_schedule')
    if ss:
        print(' serial', ss['ms_per_step'], {x: round(v['ms'] / ss['steps'], 3) for x, v in ss['phases_ms_total'].items()
                                           if x.split('/')[-1].startswith('msm_')})
    if m:
        print(' msm_g1 phases', m['roofline']['phase_ms'])
    if d.get('cpu_baseline'):
        print(' cpu', d['cpu_baseline']['value'])
