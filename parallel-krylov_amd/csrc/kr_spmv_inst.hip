// Kernel instantiations of ONE SpMV epilogue (KR_EPI = SpmvEpi value), built
// once per epilogue by the Makefile so the variants compile in parallel.
#include "kr_spmv.h"

#ifndef KR_EPI
#error "build with -DKR_EPI=<SpmvEpi value>"
#endif

namespace kr {
template void spmv_launch_epi<KR_EPI>(const SpmvArgs& a, int nblocks, hipStream_t s);
}  // namespace kr
