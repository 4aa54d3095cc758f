"""Round-6 summary of bench detail files (tuning)."""
import json
import sys
for f in sys.argv[1:]:
    d = json.load(open(f))
    a = d['strong_scaling_anchor']
    print(f)
    print(' prove', d['ms_per_step'], 'bit_exact', d.get('bit_exact_vs_oracle'), 'pcie+', d['pcie_inclusive']['over_resident_ms'],
          'ntt', d['ntt']['ms_per_ntt'], 'msm_g1', d['msm_g1']['ms_per_msm'], d['msm_g1']['plain']['ms_per_msm'],
          d['msm_g1']['bits64']['ms_per_msm'], 'roof', d['roofline']['frac'], d['roofline']['avg_launch_ms'],
          d['roofline']['valu']['frac'])
    print(' anchor', a['ms_per_step'], 'msm_only', a['msm_only']['ms_per_step'], a['bit_exact_vs_oracle'], 'c16',
          a['same_plan_c16']['msm_only']['ms_per_step'], a['same_plan_c16']['ms_per_step'])
    s = a.get('shard8_msm_only')
    if s:
        print(' shard', s['ms_per_step'], s['phases_ms_slowest'], s['msm_scaling_projected'], s['folded_proof_bit_exact_vs_anchor'],
              s.get('per_shard_ms'))
    ss = d['serial_schedule']
    print(' serial', ss['ms_per_step'], {x: round(v['ms'] / ss['steps'], 3) for x, v in ss['phases_ms_total'].items()
                                       if x.split('/')[-1].startswith('msm_')})
    print(' msm_g1 phases', d['msm_g1']['roofline']['phase_ms'])
    print(' cpu', d['cpu_baseline']['value'] if d.get('cpu_baseline') else None)
