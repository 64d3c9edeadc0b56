// photon_io.hip — device-side helpers of the photon file contract (SURVEY.md
// §8f row 1): pm_photons_quantize applies the %.6f text round trip in memory
// (quantize6, pm_device.hpp), so a one-process run reproduces the two-process
// reference pipeline bit for bit without writing and parsing the text.
#include "pm_internal.hpp"

namespace pmd {

__global__ void k_quantize(pm_photon* ph, int64_t n) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  pm_photon p = ph[i];
  p.pos = {quantize6(p.pos.x), quantize6(p.pos.y), quantize6(p.pos.z)};
  p.dir = {quantize6(p.dir.x), quantize6(p.dir.y), quantize6(p.dir.z)};
  p.color = {quantize6(p.color.x), quantize6(p.color.y), quantize6(p.color.z)};
  p.power = 0;   // not written to the text file: the reader leaves it zero
  ph[i] = p;
}

hipError_t photons_quantize(pm_photon* ph, int64_t n, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  k_quantize<<<grid_for(n, 256), 256, 0, s>>>(ph, n);
  PM_HIP_TRY(hipGetLastError());
  return hipStreamSynchronize(s);
}

}  // namespace pmd
