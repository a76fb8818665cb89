// kernels.h -- host-side launchers for the gfx950 kernels (kernels.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace cmtv {

constexpr uint32_t kBtabWords = 128 * 36;   // (1..128)B, 36 words per row
constexpr uint32_t kAtabWordsPerLane = 320; // (1..8)(-A), 40 words per point

hipError_t launch_btab_init(uint32_t* d_rows, hipStream_t s);
hipError_t launch_verify(uint32_t mode, uint32_t n, const void* pk, const void* sig, const void* msg,
                         const void* off, const uint32_t* btab, uint32_t* atab, void* valid, void* bitmap,
                         bool quad, hipStream_t s);
hipError_t launch_pubkey(uint32_t n, const void* seeds, const uint32_t* btab, void* out_pk, hipStream_t s);
hipError_t launch_sign(uint32_t n, const void* seeds, const void* key_idx, const void* msg, const void* off,
                       const uint32_t* btab, void* out_sig, hipStream_t s);

}  // namespace cmtv
