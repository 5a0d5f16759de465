// cv_sort.hip — the one library primitive the path uses: rocPRIM's radix sort of 64-bit
// keys, for the per-map walks of conntrack admission (cv_kernels.hip "conntrack
// admission": the packets with creates or deletes sorted by (map, packet)).  Its own
// translation unit so the rocPRIM headers compile once, apart from the kernels.
#include <rocprim/device/device_radix_sort.hpp>

#include "cv_dp.hpp"

namespace cv {

int sort_keys64(void *tmp, size_t *bytes, const unsigned long long *in, unsigned long long *out, uint32_t n,
                int end_bit, hipStream_t s)
{
    const hipError_t e = rocprim::radix_sort_keys(tmp, *bytes, in, out, n, 0u, (unsigned)end_bit, s);
    return e == hipSuccess ? 0 : -EIO;
}

}  // namespace cv
