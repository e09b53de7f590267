// fp32 -> zero-padded bf16 operand copy (cast_pad_kernel, csrc/norm.hip; also the packing launch of the fused
// transformer, csrc/tr_ffn.hip frag_pack_kernel): rows past `rows` and columns past `cols` are written as zeros
#pragma once
#include "common.h"

struct CastItem {
  const float* src;
  __bf16* dst;
  int rows, cols, rows_p, cols_p, ld_src;
};

// one item over blocks bx of nbx (blockDim.x threads each): 8 consecutive columns per thread (16-B bf16 store; two
// 16-B loads when the source row allows), 32-bit index math
__device__ __forceinline__ void cast_item_run(const CastItem& it, int bx, int nbx) {
  if ((it.cols_p & 7) == 0 && (long)it.rows_p * it.cols_p < (1L << 31)) {
    const int c8 = it.cols_p >> 3;
    const int total = it.rows_p * c8;
    const bool vsrc = (it.ld_src & 3) == 0 && (((uintptr_t)it.src) & 15) == 0;
    for (int e = bx * blockDim.x + threadIdx.x; e < total; e += nbx * blockDim.x) {
      const int r = e / c8, c = (e - r * c8) * 8;
      float v[8];
      if (r < it.rows && vsrc && c + 8 <= it.cols) {
        const float4 x0 = *reinterpret_cast<const float4*>(it.src + (size_t)r * it.ld_src + c);
        const float4 x1 = *reinterpret_cast<const float4*>(it.src + (size_t)r * it.ld_src + c + 4);
        v[0] = x0.x; v[1] = x0.y; v[2] = x0.z; v[3] = x0.w; v[4] = x1.x; v[5] = x1.y; v[6] = x1.z; v[7] = x1.w;
      } else {
#pragma unroll
        for (int k = 0; k < 8; ++k) v[k] = (r < it.rows && c + k < it.cols) ? it.src[(size_t)r * it.ld_src + c + k] : 0.f;
      }
      bf16x8 o;
#pragma unroll
      for (int k = 0; k < 8; ++k) o[k] = (__bf16)v[k];
      *reinterpret_cast<bf16x8*>(it.dst + (size_t)r * it.cols_p + c) = o;
    }
    return;
  }
  const long total = (long)it.rows_p * it.cols_p;
  for (long e = (long)bx * blockDim.x + threadIdx.x; e < total; e += (long)nbx * blockDim.x) {
    const int r = (int)(e / it.cols_p), c = (int)(e % it.cols_p);
    const float v = (r < it.rows && c < it.cols) ? it.src[(size_t)r * it.ld_src + c] : 0.f;
    it.dst[e] = (__bf16)v;
  }
}
