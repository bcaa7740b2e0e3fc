// Launch geometry shared by the HIP kernels.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace dglhip {

// The grid size of one dimension is limited to 2^32 - 1 work-items: 2^26 rows
// at one 64-lane wave each (RMAT-26) with four waves per 256-lane block is
// already 2^32. Large 1-D launches are folded into a 2-D grid, x fastest, so
// the dispatch order is still the linear block order (the degree-descending
// row schedule). Blocks past the end exit on the kernels' bounds checks.
constexpr int64_t kGridX = int64_t(1) << 16;

inline dim3 grid_1d(int64_t blocks) {
  if (blocks <= kGridX) return dim3(static_cast<unsigned>(blocks));
  return dim3(static_cast<unsigned>(kGridX), static_cast<unsigned>((blocks + kGridX - 1) / kGridX));
}

__device__ __forceinline__ int64_t block_linear() {
  return int64_t(blockIdx.y) * int64_t(gridDim.x) + int64_t(blockIdx.x);
}

}  // namespace dglhip
