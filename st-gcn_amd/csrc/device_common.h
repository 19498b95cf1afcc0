// Device helpers shared by the fp32 (kernels.hip) and bf16 (kernels_bf16.hip)
// GEMM kernels of libstgcn_hip.so. gfx950 only.
#pragma once
#include <hip/hip_runtime.h>

#include <type_traits>

#include "internal.h"

namespace stgcn {

typedef float floatx16 __attribute__((ext_vector_type(16)));

__device__ __forceinline__ floatx16 mfma32(float a, float b, floatx16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__device__ __forceinline__ float wave_sumf(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// Block (NT threads) reduction of two doubles, then one fp64 atomic each.
// `red` must hold 2*NT/64 doubles of LDS.
template <int NT>
__device__ __forceinline__ void block_sum2_atomic(double a, double b, double *dst_a,
                                                  double *dst_b, double *red) {
  a = wave_sum(a);
  b = wave_sum(b);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  if (lane == 0) {
    red[w] = a;
    red[NT / 64 + w] = b;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    double sa = 0.0, sb = 0.0;
    for (int i = 0; i < NT / 64; ++i) {
      sa += red[i];
      sb += red[NT / 64 + i];
    }
    atomicAdd(dst_a, sa);
    if (dst_b) atomicAdd(dst_b, sb);
  }
  __syncthreads();
}

// LDS-DMA through a buffer resource: LDS[lds_wave_base + lane] = base[voff/4]
// for this lane's byte offset; offsets >= the resource's size (kOOB) return 0,
// which zero-fills the temporal halo and all padding without branches.
// lds_wave_base must be the same for the whole wave.
constexpr unsigned kOOB = 0x80000000u;

__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const float *base, int64_t nfloats) {
  int64_t bytes = nfloats * 4;
  if (bytes > 0x7fffffffLL) bytes = 0x7fffffffLL;
  return __builtin_amdgcn_make_buffer_rsrc((void *)base, 0, (int)bytes, 0x00020000);
}

__device__ __forceinline__ void blds_f32(__amdgpu_buffer_rsrc_t rs, unsigned voff,
                                         float *lds_wave_base) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, lds_wave_base, 4, voff, 0, 0, 0);
}

__host__ __device__ constexpr int round64(int x) { return (x + 63) & ~63; }

// XCD-aware bijective remap: hardware deals consecutive block ids round-robin
// over the 8 XCDs; give each XCD a contiguous chunk of the logical grid so
// workgroups that share input tiles share an L2 (speed only, never correctness).
__device__ __forceinline__ int xcd_remap(int bid, int nblk) {
  const int q = nblk / 8, r = nblk % 8;
  const int xcd = bid % 8, loc = bid / 8;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + loc;
}

// Epilogue of a conv tile (k_tconv, k_conv_bf16): 64 rows x NCOLS (<= 256)
// columns = (NCOLS / V) frames, held as 4 32x32 fp32 MFMA accumulators per
// wave (wave w: rows (w&1)*32..+31, column tiles (w>>1)*4..+3; the C/D layout
// is the same for v_mfma_f32_32x32x2_f32 and v_mfma_f32_32x32x16_bf16).
// Adds the biases, the residual, ReLU and dropout, stores, and accumulates the
// per-row BN statistics (fp64). smem: >= 2 KiB of LDS no wave reads any more
// (BV_LDS: + 64*V floats; the tile's rows of the bias table bias_rv are staged
// there by coalesced loads instead of one scattered load per element).
template <int V, int NCOLS, bool BV_LDS = false>
__device__ __forceinline__ void conv_tile_epilogue(const ConvGemmParams &p, floatx16 (&acc)[4],
                                                   int n, int r0, int m0, float *smem) {
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int hi = lane >> 5, lo = lane & 31;
  const int mi = wave & 1, nj0 = (wave >> 1) * 4;
  // Epilogue: bias, store, optional per-row BN statistics (fp64). Buffer
  // loads/stores with 32-bit offsets; masked elements get offset kOOB (loads
  // return 0, stores are dropped), so there is no per-element branch.
  const int ostride = p.T_dst * V;
  const __amdgpu_buffer_rsrc_t rs_o = make_rsrc(p.out + (int64_t)n * p.out_bstride, p.out_bstride);
  const __amdgpu_buffer_rsrc_t rs_b = make_rsrc(p.bias_r ? p.bias_r : p.out, p.bias_r ? p.R : 0);
  const __amdgpu_buffer_rsrc_t rs_bv =
      make_rsrc(p.bias_rv ? p.bias_rv : p.out, p.bias_rv ? (int64_t)p.R * V : 0);
  float *sbv = smem + 512;  // past the statistics partials (2 KiB)
  if constexpr (BV_LDS) {
    if (p.bias_rv) {  // uniform
      const int nrow = min(64, p.R - r0);
      for (int i = tid; i < nrow * V; i += blockDim.x) sbv[i] = p.bias_rv[r0 * V + i];
      __syncthreads();
    }
  }
  const __amdgpu_buffer_rsrc_t rs_res = make_rsrc(
      p.res ? p.res + (int64_t)n * p.out_bstride : p.out, p.res ? p.out_bstride : 0);
  int ocol[4], cv[4];
  bool cok[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int col = (nj0 + j) * 32 + lo;
    const int mf = col / V;
    const int v = col - mf * V;
    const int m = m0 + mf;
    cok[j] = col < NCOLS && m < p.M;
    cv[j] = v;
    ocol[j] = (p.s_out * m + p.p_out) * V + v;
  }
  const int rowb = r0 + mi * 32 + 4 * hi;
  auto epilogue = [&](auto stats_c) {
    constexpr bool STATS = decltype(stats_c)::value;
    double *red = reinterpret_cast<double *>(smem);  // [4 waves][2 halves][32]
#pragma unroll
    for (int g = 0; g < 4; ++g) {  // groups of 4 accumulator registers
      double gv[8];                // [stat][register]: partials over this lane's 4 columns
#pragma unroll
      for (int ii = 0; ii < 4; ++ii) {
        const int i = g * 4 + ii;
        const int row = rowb + (i & 3) + 8 * (i >> 2);
        const bool rok = row < p.R;
        const float br = __builtin_bit_cast(
            float, __builtin_amdgcn_raw_buffer_load_b32(rs_b, rok ? row * 4 : (int)kOOB, 0, 0));
        double s = 0.0, sq = 0.0;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const bool ok = rok && cok[j];
          float val = acc[j][i] + br;
          if constexpr (BV_LDS) {
            if (p.bias_rv && ok) val += sbv[(row - r0) * V + cv[j]];
          } else {
            val += __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(
                                                 rs_bv, ok ? (row * V + cv[j]) * 4 : (int)kOOB, 0, 0));
          }
          const int off = ok ? (row * ostride + ocol[j]) * 4 : (int)kOOB;
          if (p.res)
            val += __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rs_res, off, 0, 0));
          if (p.relu_out) val = fmaxf(val, 0.f);
          if (p.drop.thresh && ok)
            val = dropout_keep(p.drop, (uint64_t)n * p.out_bstride + row * ostride + ocol[j])
                      ? val * p.drop.scale
                      : 0.f;
          __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, val), rs_o, off, 0, 0);
          if constexpr (STATS) {
            const double dv = ok ? (double)val : 0.0;
            s += dv;
            sq += dv * dv;
          }
        }
        gv[ii] = s;
        gv[4 + ii] = sq;
      }
      if constexpr (STATS) {
        // butterfly over the 32 lanes of the wave half (fp64): reduce-scatter
        // the 8 values over lane bits 4, 3, 2, then all-reduce over bits 1, 0;
        // lane lo ends with value (lo >> 2) = stat*4 + register-in-group
#pragma unroll
        for (int h = 16, n = 8; h >= 4; h >>= 1, n >>= 1) {
          const bool up = lo & h;
#pragma unroll
          for (int v = 0; v < n / 2; ++v) {
            const double send = up ? gv[v] : gv[v + n / 2];
            const double keep = up ? gv[v + n / 2] : gv[v];
            gv[v] = keep + __shfl_xor(send, h, 64);
          }
        }
        gv[0] += __shfl_xor(gv[0], 2, 64);
        gv[0] += __shfl_xor(gv[0], 1, 64);
        if ((lo & 3) == 0) red[(wave * 2 + hi) * 32 + g * 8 + (lo >> 2)] = gv[0];
      }
    }
    if constexpr (STATS) {
      __syncthreads();
      if (tid < 128) {
        const int rl = tid >> 1, sqf = tid & 1;  // tile row, statistic
        const int m = rl >> 5, rr = rl & 31;
        const int h = (rr >> 2) & 1, i = (rr & 3) + 4 * (rr >> 3);
        const int k = (i >> 2) * 8 + sqf * 4 + (i & 3);
        const double tot = red[(m * 2 + h) * 32 + k] + red[((m + 2) * 2 + h) * 32 + k];
        const int row = r0 + rl;
        if (row < p.R) atomicAdd((sqf ? p.stat_sq : p.stat_sum) + row, tot);
      }
    }
  };
  if (p.stat_sum)
    epilogue(std::true_type{});
  else
    epilogue(std::false_type{});
}

}  // namespace stgcn
