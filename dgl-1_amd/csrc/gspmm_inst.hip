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

#if GSPMM_INST_MSG == 0 && GSPMM_INST_EM == 1  // copy_u, scalar layout: the headline kernel
extern "C" int dglhip_gspmm_resident_waves(int device, int64_t* waves) {
  API_BEGIN();
  using namespace dglhip;
  DGLHIP_CHECK(waves != nullptr, "null pointer argument");
  int cus = 0, blocks = 0;
  HIP_CALL(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device));
  // the F = 128 copy_u + sum kernel (2 floats x 64 lanes, 16 gathers in flight)
  HIP_CALL(hipOccupancyMaxActiveBlocksPerMultiprocessor(
      &blocks,
      reinterpret_cast<const void*>(
          &gspmm_sum_kernel<2, 64, 16, DGLHIP_MSG_COPY_U, EM_SCALAR, false, false, false>),
      256, 0));
  *waves = int64_t(cus) * blocks * 4;  // 256-lane blocks: 4 waves each
  API_END();
}
#endif
