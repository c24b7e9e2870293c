"""Instruction counts and register usage of one kernel in a hipcc --save-temps .s file.
usage: asm_stats.py file.s kernel_symbol_prefix [--loop]"""
import re
import sys

S, pref = sys.argv[1], sys.argv[2]
lines = open(S).read().split('\n')
start = [i for i, l in enumerate(lines) if l.startswith(pref) and ':' in l][0]
end = [i for i in range(start, len(lines)) if lines[i].startswith('.Lfunc_end')][0]
body = lines[start:end]
print(lines[start].split(':')[0], "lines", len(body))
for k in ['v_mfma', 's_barrier', 's_waitcnt', 'global_load_lds', 'ds_read_b128', 'ds_write', 'scratch_',
          's_cbranch', 'global_store', 'global_load_dword', 'v_exp', 'v_rcp', 's_setprio']:
    print(f"  {k:18s} {sum(1 for l in body if k in l)}")
txt = open(S).read()
sym = lines[start].split(':')[0]
i = txt.find('.name:           ' + sym)
m = txt[txt.rfind('.agpr_count', 0, i) - 10:i]
for l in m.split('\n'):
    if any(k in l for k in ['agpr_count', 'sgpr_count', 'vgpr_count', 'spill', 'group_segment']):
        print("  " + l.strip())
if '--waits' in sys.argv:
    for j, l in enumerate(body):
        if 's_waitcnt' in l or 's_barrier' in l:
            print(j, l.strip())
