import shutil
import os
src = os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', '..', '..', 'tfg---quantum-byzantine-agreement_amd', 'csrc')
name='t_ts'
dst = f'/tmp/c1v/{name}/csrc'
shutil.rmtree(f'/tmp/c1v/{name}', ignore_errors=True)
shutil.copytree(src, dst)
p = dst + '/qba_lists_kern.h'; s = open(p).read()
# global stamp buffer
a = '''template <int NP>
struct QCfg {'''
b = '''__device__ unsigned long long g_qba_ts[4096 * 4];
template <int NP>
struct QCfg {'''
assert s.count(a) == 1; s = s.replace(a, b, 1)
# stage end stamp (first __syncthreads in qba_lists_body)
a = '''    for (int i = threadIdx.x; i < NZ; i += BS) hist[i] = 0u;
  }
  __syncthreads();'''
b = '''    for (int i = threadIdx.x; i < NZ; i += BS) hist[i] = 0u;
  }
  __syncthreads();
  if (threadIdx.x == 0) g_qba_ts[blockIdx.x * 4 + 1] = __builtin_amdgcn_s_memrealtime();'''
assert s.count(a) == 1, 'stage'; s = s.replace(a, b)
a = '''  if (MODE != 0) {
    __syncthreads();
    uint32_t *row = slab + (size_t)bid * C::NBP;'''
b = '''  if (MODE != 0) {
    __syncthreads();
    if (threadIdx.x == 0) g_qba_ts[blockIdx.x * 4 + 2] = __builtin_amdgcn_s_memrealtime();
    uint32_t *row = slab + (size_t)bid * C::NBP;'''
assert s.count(a) == 1, 'main'; s = s.replace(a, b)
a = '''  extern __shared__ __align__(16) uint64_t lds[];
  const uint32_t nl = gridDim.x - (uint32_t)d.red;
  if (blockIdx.x >= nl) {  // workgroup-uniform
    constexpr int NP4 = qba_def_parts<NP>();
    const int r = (int)(blockIdx.x - nl);
    qba_reduce_u<NP>(d, r / NP4, r % NP4, (int)threadIdx.x, QBA_DBLOCK, reinterpret_cast<uint32_t *>(lds));
    return;
  }
  qba_lists_body<NP, 1, SAMP, QPT, PK, QBA_DBLOCK, 0, QBA_DEF_PAIRWISE>(ps, k0, k1, first, count, lists,
                                                                                   ld, slab, zero, 0u, (uint32_t)d.red);'''
b = '''  extern __shared__ __align__(16) uint64_t lds[];
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  const uint32_t nl = gridDim.x - (uint32_t)d.red;
  if (blockIdx.x >= nl) {  // workgroup-uniform
    constexpr int NP4 = qba_def_parts<NP>();
    const int r = (int)(blockIdx.x - nl);
    qba_reduce_u<NP>(d, r / NP4, r % NP4, (int)threadIdx.x, QBA_DBLOCK, reinterpret_cast<uint32_t *>(lds));
    __syncthreads();
    if (threadIdx.x == 0) {
      g_qba_ts[blockIdx.x * 4 + 0] = t0; g_qba_ts[blockIdx.x * 4 + 1] = 0; g_qba_ts[blockIdx.x * 4 + 2] = 0;
      g_qba_ts[blockIdx.x * 4 + 3] = __builtin_amdgcn_s_memrealtime() | (1ull << 63);
    }
    return;
  }
  qba_lists_body<NP, 1, SAMP, QPT, PK, QBA_DBLOCK, 0, QBA_DEF_PAIRWISE>(ps, k0, k1, first, count, lists,
                                                                                   ld, slab, zero, 0u, (uint32_t)d.red);
  __syncthreads();
  if (threadIdx.x == 0) { g_qba_ts[blockIdx.x * 4 + 0] = t0; g_qba_ts[blockIdx.x * 4 + 3] = __builtin_amdgcn_s_memrealtime(); }'''
assert s.count(a) == 1, 'def'; s = s.replace(a, b)
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
