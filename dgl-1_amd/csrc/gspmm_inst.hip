// One (message, edge-feature layout) pair of the g-SpMM sum/mean/max kernels,
// selected by -DGSPMM_INST_MSG=<DGLHIP_MSG_*> -DGSPMM_INST_EM=<EM_*> (Makefile).
// Splitting the instantiations over translation units lets them compile in
// parallel; the kernels themselves live in gspmm_impl.h.
#include "gspmm_impl.h"

namespace dglhip {
template void dispatch_sum_me<GSPMM_INST_MSG, GSPMM_INST_EM>(bool, const SumLaunch&,
                                                             hipStream_t);
template void dispatch_max_me<GSPMM_INST_MSG, GSPMM_INST_EM>(const MaxLaunch&, hipStream_t);
}  // namespace dglhip
