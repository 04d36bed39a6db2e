import sys, shutil
import os
src = os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', '..', '..', 'tfg---quantum-byzantine-agreement_amd', 'csrc')
name, kind = sys.argv[1], sys.argv[2]
dst = f'/tmp/c1v/{name}/csrc'
shutil.rmtree(f'/tmp/c1v/{name}', ignore_errors=True)
shutil.copytree(src, dst)
p = dst + '/qba_lists_kern.h'; s = open(p).read()
if kind == 'noatomic':
    a = '''        atomicAdd((uint32_t *)((qba_lds_u32 *)(uintptr_t)a + g * C::WP), 1u);'''
    b = '''        asm volatile("" ::"v"(a));'''
    assert s.count(a) == 1; s = s.replace(a, b)
elif kind == 'nocond3':
    a = '''  // Cond3 (tfg.py:96-98): distinct iff the union of the values' 16-bit
  // one-hots (two per v_pk_lshlrev_b16) has n+1 bits
  uint32_t U = 0;'''
    b = '''  if (l1r != 0xfffu) return;
  uint32_t U = 0;'''
    assert s.count(a) == 1; s = s.replace(a, b)
elif kind == 'noloop':
    a = '''  const uint32_t nunits = count / (4 * QPT);'''
    b = '''  const uint32_t nunits = 0u * count;'''
    assert s.count(a) == 1; s = s.replace(a, b)
    a = '''  if (bid == nblk - 1 && threadIdx.x < rq) {
    const uint32_t c0 = r0 + 4 * threadIdx.x;
    if (c0 + 4 <= count)
      qba_step_l<NP, MODE, SAMP, 1, false, PK, false, CNT, PW>'''
    b = '''  if (bid == nblk - 1 && threadIdx.x < 0 * rq) {
    const uint32_t c0 = r0 + 4 * threadIdx.x;
    if (c0 + 4 <= count)
      qba_step_l<NP, MODE, SAMP, 1, false, PK, false, CNT, PW>'''
    assert s.count(a) == 1, 'tail'; s = s.replace(a, b)
open(p, 'w').write(s)
