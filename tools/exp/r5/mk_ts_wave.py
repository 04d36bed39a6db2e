import shutil
import os
src = os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', '..', '..', 'tfg---quantum-byzantine-agreement_amd', 'csrc')
name='t_ts2'
dst = f'/tmp/c1v/{name}/csrc'
shutil.rmtree(f'/tmp/c1v/{name}', ignore_errors=True)
shutil.copytree(src, dst)
p = dst + '/qba_lists_kern.h'; s = open(p).read()
a = '''template <int NP>
struct QCfg {'''
b = '''__device__ unsigned long long g_qba_ts[4096 * 16][8];
#define QBA_TS(i) do { if ((threadIdx.x & 63) == 0) g_qba_ts[blockIdx.x * 16 + (threadIdx.x >> 6)][i] = __builtin_amdgcn_s_memrealtime(); } while (0)
template <int NP>
struct QCfg {'''
assert s.count(a) == 1; s = s.replace(a, b, 1)
# stamps in qba_step_pk MODE 1 (sample branch)
a = '''    for (int k = 0; k < QPT; ++k) {
      qba_sample_quad<NP, SAMP, TAIL, PW>(c0 + 4 * k, valid, first, k0, k1, ps, pat, apat, thr, pl, D);
#pragma unroll
      for (int i = 0; i < ND; ++i) {
        Dp[2 * k][i] = D[0][i] | (D[1][i] << 4);'''
b = '''    for (int k = 0; k < QPT; ++k) {
      if (!TAIL && k == 0) QBA_TS(1);
      qba_sample_quad<NP, SAMP, TAIL, PW>(c0 + 4 * k, valid, first, k0, k1, ps, pat, apat, thr, pl, D);
      if (!TAIL) QBA_TS(2 + 2 * k);
#pragma unroll
      for (int i = 0; i < ND; ++i) {
        Dp[2 * k][i] = D[0][i] | (D[1][i] << 4);'''
assert s.count(a) == 1, 'pk'; s = s.replace(a, b)
a = '''    if (!TAIL && act) {
      uint64_t rbl = 0;  // the running row base'''
b = '''    if (!TAIL) QBA_TS(6);
    if (!TAIL && act) {
      uint64_t rbl = 0;  // the running row base'''
assert s.count(a) == 1, 'store'; s = s.replace(a, b)
# after pushes of quad k: stamp 3 / 5 -> place after the MODE==1 push block: find "      }\n    }\n    if (!TAIL) QBA_TS(6);"
a = '''    if (!TAIL) QBA_TS(6);'''
s = s.replace(a, a)  # keep
# main loop end and final drains
a = '''    while (wq.qn) {  // wave-uniform'''
b = '''    QBA_TS(7);
    while (wq.qn) {  // wave-uniform'''
assert s.count(a) == 1, 'drain'; s = s.replace(a, b)
a = '''  if (MODE != 0) {
    __syncthreads();
    uint32_t *row = slab + (size_t)bid * C::NBP;'''
b = '''  if (MODE != 0) {
    QBA_TS(0);
    __syncthreads();
    uint32_t *row = slab + (size_t)bid * C::NBP;'''
assert s.count(a) == 1, 'flush'; s = s.replace(a, b)
open(p, 'w').write(s)
p = dst + '/qba_lists_inst.hip'; s = open(p).read()
s += '''
#if QBA_INST_N == 11
extern "C" __attribute__((visibility("default"))) int qba_exp_ts(void *host) {
  return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(g_qba_ts), sizeof(g_qba_ts));
}
#endif
'''
open(p, 'w').write(s)
