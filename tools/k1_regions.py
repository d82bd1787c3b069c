"""Static instruction counts of zh_lz_kernel (K1, mode 0) per phase: copies csrc/zh_lz.hip to
/tmp/mk with asm comment markers (";@R name") at the phase boundaries, compiles it for gfx950
with -save-temps and counts v_ / s_ / ds_ / global_ instructions between markers in the kernel's
assembly.  Regions follow code layout (an inlined function's copies add up), so the numbers
rank phases and compare builds; the dynamic split is the perturbation study
(profiles/r05i_k1_perturbation.json).  usage: python3 tools/k1_regions.py > profiles/<tag>_k1_regions.txt"""
import os, re, subprocess, sys, collections
os.makedirs('/tmp/mk', exist_ok=True)
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
src = open(os.path.join(ROOT, 'custom-nvcomp-with-zstd_amd/csrc/zh_lz.hip')).read()
def M(name): return f'__asm__ volatile(";@R {name}");'
reps = [
 ('    loadA(k);\n', '    __asm__ volatile(";@R A");\n    loadA(k);\n'),
 ('#pragma unroll\n  for (u32 k = 0; k < MAX_RW; k++) c1(k);\n', '  __asm__ volatile(";@R C1");\n#pragma unroll\n  for (u32 k = 0; k < MAX_RW; k++) c1(k);\n'),
 ('    u32 const r = r_hi - 1 - k, i = 64 * r + lane, p = wsb + i;\n', '    __asm__ volatile(";@R C2");\n    u32 const r = r_hi - 1 - k, i = 64 * r + lane, p = wsb + i;\n'),
 # inserter
 ('  load_in(wsb + T0 * ZH_TILE);\n', '  if constexpr (LONG) { ' + M('insL') + ' } else { ' + M('insS') + ' }\n  load_in(wsb + T0 * ZH_TILE);\n'),
 ('      insert_repair<LONG, BT>(T, tb0, lane, h, e);\n', '      ' + M('repair') + '\n      insert_repair<LONG, BT>(T, tb0, lane, h, e);\n      if constexpr (LONG) { ' + M('insL') + ' } else { ' + M('insS') + ' }\n'),
 ('    if (t0 == 0 && skip) {\n      bool v = false;', '    if (t0 == 0 && skip) {\n      ' + M('rcheck') + '\n      bool v = false;'),
 ('      if (!on_check(__ballot(v) != 0)) {', '      if constexpr (LONG) { ' + M('insL') + ' } else { ' + M('insS') + ' }\n      if (!on_check(__ballot(v) != 0)) {'),
 ('  __asm__ volatile("" ::: "memory");\n}\n// The next window\'s first position', '  __asm__ volatile("" ::: "memory");\n  ' + M('insx') + '\n}\n// The next window\'s first position'),
 # span lengths
 ('  u32 olo[MAX_RW], ohi[MAX_RW], Lw[MAX_RW][3], Sw[MAX_RW][3];\n', '  ' + M('passA') + '\n  u32 olo[MAX_RW], ohi[MAX_RW], Lw[MAX_RW][3], Sw[MAX_RW][3];\n'),
 ('  if (nq) xq_flush(in32, ci, xq, nq, wsb, lane);\n', '  if (nq) xq_flush(in32, ci, xq, nq, wsb, lane);\n  ' + M('passC') + '\n'),
 ('    if (lane == 0) tm[r] = tb;\n  }\n}\n', '    if (lane == 0) tm[r] = tb;\n  }\n  ' + M('spanx') + '\n}\n'),
 ('  bool const act = lane < k;\n  u32 const e = act ? xq[lane] : 0u;', '  ' + M('flush') + '\n  bool const act = lane < k;\n  u32 const e = act ? xq[lane] : 0u;'),
 ('  if (act) ((u8 *)ci)[4 * cidx(i) + (sh >> 3)] = (u8)x;\n}', '  if (act) ((u8 *)ci)[4 * cidx(i) + (sh >> 3)] = (u8)x;\n  ' + M('passA') + '\n}'),
 # walk
 ('      seg_walk<false>(ciP, tmk, S, SE, entry, true, LM, MM, ex);\n', '      ' + M('walk') + '\n      seg_walk<false>(ciP, tmk, S, SE, entry, true, LM, MM, ex);\n'),
 ('      e_in = wsp + lane_value(ex, 63);\n', '      e_in = wsp + lane_value(ex, 63);\n      ' + M('mlist') + '\n'),
 ('    if (wave == REC_WAVE && prev2) {\n', '    ' + M('rec') + '\n    if (wave == REC_WAVE && prev2) {\n'),
 ('    if (lane == 0) atomicAdd(&misc[MISC_ARR], 1u);\n    k1_barrier();  // X', '    ' + M('X') + '\n    if (lane == 0) atomicAdd(&misc[MISC_ARR], 1u);\n    k1_barrier();  // X'),
 ('    if (prev2) {\n      // ---- literals of window k - 2', '    ' + M('lits') + '\n    if (prev2) {\n      // ---- literals of window k - 2'),
 ('    ZH_STAMP(st_E);\n  }\n  if (!dead) {', '    ZH_STAMP(st_E);\n    ' + M('loop') + '\n  }\n  if (!dead) {'),
 ('    bool const skipk = have && skip_window_eff(misc, k, kskip0);\n', '    ' + M('steptop') + '\n    bool const skipk = have && skip_window_eff(misc, k, kskip0);\n'),
 ('  if (repeat_scan(in32, (u32 *)TL, hw, misc, pre, n, tid)) return K1_REDO;\n#endif\n', '  ' + M('scan') + '\n  if (repeat_scan(in32, (u32 *)TL, hw, misc, pre, n, tid)) return K1_REDO;\n#endif\n  ' + M('dead') + '\n'),
 ('  ZH_STAMP(st_stage);\n', '  ZH_STAMP(st_stage);\n  ' + M('prologue_end') + '\n'),
]
for a, b in reps:
    if a not in src: print('MISSING', a[:60]); sys.exit(1)
    src = src.replace(a, b, 1)
open('/tmp/mk/zh_lz.hip', 'w').write(src)
subprocess.check_call('cd /tmp/mk && /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -I' + ROOT + '/include -I' + ROOT + '/custom-nvcomp-with-zstd_amd/csrc -c zh_lz.hip -o x.o -save-temps 2>/dev/null', shell=True)
asm = open('/tmp/mk/zh_lz-hip-amdgcn-amd-amdhsa-gfx950.s').read().split('\n')
fn = sys.argv[1] if len(sys.argv) > 1 else 'zh_lz_kernel'
i0 = asm.index(f'{fn}:' + ' ' * (41 - len(fn) - 1 - 0) if False else None) if False else None
start = next(i for i, l in enumerate(asm) if l.startswith(fn + ":"))
end = next(i for i in range(start, len(asm)) if asm[i].startswith(".Lfunc_end"))
cnt = collections.Counter(); cur = 'pre'
for l in asm[start:end]:
    t = l.strip()
    m = re.match(r';@R (\S+)', t)
    if not m and t.startswith(';@R'): m = re.match(r';@R\s*(\S+)', t)
    if m: cur = m.group(1); continue
    if not t or t.startswith(';') or t.startswith('.') or t.endswith(':'): continue
    op = t.split()[0]
    if op.startswith('v_'): cnt[(cur, 'v')] += 1
    elif op.startswith('s_'): cnt[(cur, 's')] += 1
    elif op.startswith('ds_'): cnt[(cur, 'ds')] += 1
    elif op.startswith('global_') or op.startswith('buffer_') or op.startswith('flat_'): cnt[(cur, 'g')] += 1
regs = sorted(set(k[0] for k in cnt))
for r in regs: print(f'{r:14s} v {cnt[(r,"v")]:5d}  s {cnt[(r,"s")]:5d}  ds {cnt[(r,"ds")]:4d}  g {cnt[(r,"g")]:4d}')
