// Kernel instantiations of ONE SpMV epilogue (KR_EPI = SpmvEpi value), built
// once per epilogue by the Makefile so the variants compile in parallel.
#include "kr_spmv.h"

#ifndef KR_EPI
#error "build with -DKR_EPI=<SpmvEpi value>"
#endif

namespace kr {
template void spmv_launch_epi<KR_EPI>(const SpmvArgs& a, int nblocks, hipStream_t s);
#if KR_EPI == 7
static_assert(EPI_DUAL_MRR == 7, "the fused basis pair is built with EPI_DUAL_MRR's unit");
void launch_spmv_stencil2(const SpmvArgs& a, int nblocks, hipStream_t s) {
  spmv_stencil2_launch(a, nblocks, s);
}
#endif
#if KR_EPI == 7
void launch_spmv_stencil2t_mrr(const SpmvArgs& a, int nblocks, hipStream_t s) {
  spmv_stencil2t_launch<EPI_DUAL_MRR>(a, nblocks, s);
}
#endif
#if KR_EPI == 8
static_assert(EPI_DUAL_KCG == 8, "the tiled pair's k-skip CG products are built in EPI_DUAL_KCG's unit");
void launch_spmv_stencil2t_kcg(const SpmvArgs& a, int nblocks, hipStream_t s) {
  spmv_stencil2t_launch<EPI_DUAL_KCG>(a, nblocks, s);
}
#endif
}  // namespace kr
