"""Summary of SQ counter passes (tools/gpu_round_pmc.sh): usage: sq_summary.py <dir> <label> [<dir> <label> ...]"""
import csv, glob, sys, collections
for d, envs in zip(sys.argv[1::2], sys.argv[2::2]):
    acc = collections.defaultdict(lambda: collections.defaultdict(float)); disp = collections.defaultdict(set)
    for f in glob.glob(d + '/**/*counter_collection.csv', recursive=True):
        for r in csv.DictReader(open(f)):
            k = r['Kernel_Name']
            if 'fdk::' not in k: continue
            k = k.replace('void ', '').replace('fdk::(anonymous namespace)::', '').split('(')[0]
            acc[k][r['Counter_Name']] += float(r['Counter_Value']); disp[k].add(r['Dispatch_Id'])
    for k, c in acc.items():
        n = len(disp[k]); c = {a: b / n for a, b in c.items()}
        cyc = c['GRBM_GUI_ACTIVE'] / 8
        simd_instr = c['SQ_INSTS_VALU'] / 1024
        print(f"{envs:44s} {k:40s} VALU_instr={c['SQ_INSTS_VALU']/1e6:.1f}M dual_issue_quads={c['SQ_ACTIVE_INST_VALU2']/1e6:.1f}M "
              f"kernel_cycles={cyc/1e6:.3f}M cycles/VALU_instr/SIMD={cyc/simd_instr:.2f} "
              f"slot_busy={(simd_instr - c['SQ_ACTIVE_INST_VALU2']/1024)*4/cyc:.2f} waves/SIMD={c['SQ_WAVE_CYCLES']*4/1024/cyc:.2f} "
              f"issue_stalled={c['SQ_WAIT_INST_ANY']/c['SQ_WAVE_CYCLES']:.2f} waitcnt={c['SQ_WAIT_ANY']/c['SQ_WAVE_CYCLES']:.2f}")
