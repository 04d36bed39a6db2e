import sys, shutil
import os
src = os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', '..', '..', 'tfg---quantum-byzantine-agreement_amd', 'csrc')
name, pw, waves = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
dst = f'/tmp/c1v/{name}/csrc'
shutil.rmtree(f'/tmp/c1v/{name}', ignore_errors=True)
shutil.copytree(src, dst)
p = dst + '/qba_internal.h'; s = open(p).read()
s = s.replace('#define QBA_DBLOCK 768 ', '#define QBA_DBLOCK 1024 ')
open(p, 'w').write(s)
p = dst + '/qba_lists_kern.h'; s = open(p).read()
s = s.replace('constexpr int QBA_DEF_PAIRWISE = 0;', f'constexpr int QBA_DEF_PAIRWISE = {pw};')
s = s.replace('constexpr int QBA_DEF_WAVES = 6;', f'constexpr int QBA_DEF_WAVES = {waves};')
a = '''  (L.packed ? (wide ? (const void *)qba_k_lists_def<NP, S, 2, 1> : (const void *)qba_k_lists_def<NP, S, 1, 1>) \\'''
b = '''  (L.packed ? ((wide && L.count > (1u << 22)) ? (const void *)qba_k_lists_def<NP, S, 2, 1> : (const void *)qba_k_lists_def<NP, S, 1, 1>) \\'''
assert s.count(a) == 1; s = s.replace(a, b)
a = '''    dgrid = grid_for(ctx, kd, dlds, L.count, wide ? (L.packed ? 2 : QBA_GRID_QPT) : 1, &dcap, QBA_DBLOCK);'''
b = '''    dgrid = grid_for(ctx, kd, dlds, L.count, wide ? (L.packed ? (L.count > (1u << 22) ? 2 : 1) : QBA_GRID_QPT) : 1, &dcap, QBA_DBLOCK);'''
assert s.count(a) == 1; s = s.replace(a, b)
open(p, 'w').write(s)
