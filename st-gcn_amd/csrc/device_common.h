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

// Operand bounds of the fp16-split GEMMs (f16x2): max |x| as float bits
// (non-negative floats order as unsigned integers) in kAmaxSlots words
// kAmaxStride apart (one per 128-byte line), zeroed by the caller; producers
// add one atomicMax per workgroup to slot blockIdx % kAmaxSlots (thousands of
// workgroups on ONE word serialise in L2: 3.4 ms per cfg2 step measured),
// readers take the max over the slots (amax_read).

__device__ __forceinline__ unsigned amax_read(const unsigned *amax) {
  unsigned m = 0;
#pragma unroll 8
  for (int i = 0; i < kAmaxSlots; ++i) m = max(m, amax[i * kAmaxStride]);
  return m;
}

// amax_read for a whole wave (every lane active): one slot per lane and a
// shuffle max -- 1 load per lane instead of kAmaxSlots (the per-element weight
// packs read the bound once per element)
__device__ __forceinline__ unsigned amax_read_wave(const unsigned *amax) {
  static_assert(kAmaxSlots == 64, "one slot per lane");
  unsigned m = amax[(threadIdx.x & 63) * kAmaxStride];
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) m = max(m, (unsigned)__shfl_xor((int)m, o, 64));
  return m;
}

// Block (NT threads) max of m >= 0 into amax's slot of this workgroup; every
// thread of the block must call it (one barrier).
template <int NT>
__device__ __forceinline__ void block_amax(float m, unsigned *amax) {
  __shared__ float wmax[NT / 64];
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
  if ((threadIdx.x & 63) == 0) wmax[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x == 0) {
    float b = wmax[0];
#pragma unroll
    for (int i = 1; i < NT / 64; ++i) b = fmaxf(b, wmax[i]);
    const unsigned blk = blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z);
    atomicMax(amax + (blk % kAmaxSlots) * kAmaxStride, __builtin_bit_cast(unsigned, b));
  }
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
// OB: the kernel may write a bf16 output (p.out_bf16 read at run time; kept a
// template switch so the fp32-only kernels' epilogue code is unchanged)
// PF: the loads software-pipelined ahead of the stores (below; one-workgroup-
// per-CU kernels only: +72 registers)
template <int V, int NCOLS, bool BV_LDS = false, bool OB = false, bool PF = false>
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
  // (out_bf16: a resource over the bf16 tensor, byte offsets halved at the store)
  const bool ob = OB && p.out_bf16;
  const __amdgpu_buffer_rsrc_t rs_o =
      ob ? make_rsrc(reinterpret_cast<const float *>(reinterpret_cast<const __bf16 *>(p.out) +
                                                     (int64_t)n * p.out_bstride),
                     (p.out_bstride + 1) / 2)
         : make_rsrc(p.out + (int64_t)n * p.out_bstride, p.out_bstride);
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
      p.res ? p.res + (p.res_shared ? 0 : (int64_t)n * p.out_bstride) : p.out,
      p.res ? p.out_bstride : 0);
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
  // The loads of a group of 4 accumulator registers (row bias, bias table,
  // residual) are issued before the previous group's stores (software
  // pipelined): vmcnt counts loads and stores in one in-order counter, so a load
  // issued after a store can only be waited for together with that store
  struct Pre {
    float br[4], bv[16], rs[16];
  };
  auto prefetch = [&](int g, Pre &P) {
#pragma unroll
    for (int ii = 0; ii < 4; ++ii) {
      const int i = g * 4 + ii;
      const int row = rowb + (i & 3) + 8 * (i >> 2);
      const bool rok = row < p.R;
      // (null bias pointers: uniform branches, so no load is issued for them --
      // an OOB load still costs a trip through the memory pipeline and a wait)
      P.br[ii] = 0.f;
      if (p.bias_r)
        P.br[ii] = __builtin_bit_cast(
            float, __builtin_amdgcn_raw_buffer_load_b32(rs_b, rok ? row * 4 : (int)kOOB, 0, 0));
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const bool ok = rok && cok[j];
        P.bv[ii * 4 + j] = 0.f;
        P.rs[ii * 4 + j] = 0.f;
        if (!BV_LDS && p.bias_rv)
          P.bv[ii * 4 + j] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(
                                                           rs_bv, ok ? (row * V + cv[j]) * 4 : (int)kOOB, 0, 0));
        if (p.res)
          P.rs[ii * 4 + j] = __builtin_bit_cast(
              float, __builtin_amdgcn_raw_buffer_load_b32(
                         rs_res, ok ? (row * ostride + ocol[j]) * 4 : (int)kOOB, 0, 0));
      }
    }
  };
  auto epilogue = [&](auto stats_c) {
    constexpr bool STATS = decltype(stats_c)::value;
    double *red = reinterpret_cast<double *>(smem);  // [4 waves][2 halves][32]
    Pre pf[PF ? 2 : 1];
    if constexpr (PF) prefetch(0, pf[0]);
#pragma unroll
    for (int g = 0; g < 4; ++g) {  // groups of 4 accumulator registers
      if constexpr (PF)
        if (g + 1 < 4) prefetch(g + 1, pf[(g + 1) & 1]);
      const Pre &P = pf[PF ? (g & 1) : 0];
      double gv[8];                // [stat][register]: partials over this lane's 4 columns
#pragma unroll
      for (int ii = 0; ii < 4; ++ii) {
        const int i = g * 4 + ii;
        const int row = rowb + (i & 3) + 8 * (i >> 2);
        const bool rok = row < p.R;
        // (!PF: loads next to their use; null bias pointers are uniform branches,
        // so no load is issued for them)
        float br = 0.f;
        if constexpr (PF)
          br = P.br[ii];
        else if (p.bias_r)
          br = __builtin_bit_cast(
              float, __builtin_amdgcn_raw_buffer_load_b32(rs_b, rok ? row * 4 : (int)kOOB, 0, 0));
        double s = 0.0, sq = 0.0;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const bool ok = rok && cok[j];
          float val = acc[j][i] + br;
          if constexpr (BV_LDS) {
            if (p.bias_rv && ok) val += sbv[(row - r0) * V + cv[j]];
          } else if constexpr (PF) {
            val += P.bv[ii * 4 + j];
          } else if (p.bias_rv) {
            val += __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(
                                                 rs_bv, ok ? (row * V + cv[j]) * 4 : (int)kOOB, 0, 0));
          }
          const int off = ok ? (row * ostride + ocol[j]) * 4 : (int)kOOB;
          if constexpr (PF)
            val += P.rs[ii * 4 + j];
          else if (p.res)
            val += __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rs_res, off, 0, 0));
          if (p.relu_out) val = fmaxf(val, 0.f);
          if (p.drop.thresh && ok)
            val = dropout_keep(p.drop, (uint64_t)n * p.out_bstride + row * ostride + ocol[j])
                      ? val * p.drop.scale
                      : 0.f;
          if (ob)
            __builtin_amdgcn_raw_buffer_store_b16(
                __builtin_bit_cast(unsigned short, (__bf16)val), rs_o,
                ok ? (row * ostride + ocol[j]) * 2 : (int)kOOB, 0, 0);
          else
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

// ---------------------------------------------------------------------------
// Row-major epilogue for tiles staged in LDS (k_conv_x3): the workgroup's
// ROWS (64 or 128) x NCOLS tile is first written as fp32 into an LDS image [ROWS][kEpiPitch]
// (acc_to_img, one ds_write_b32 per accumulator register: lanes 0-31 and 32-63
// each write 32 consecutive words), then every thread takes whole 16-byte
// pieces of rows (TPR = NT / ROWS threads per row, piece q, q + TPR, ...) and
// applies bias / bias table / residual / ReLU / dropout / BN statistics in
// registers and stores with 16-byte stores (8- or 4-byte where the output
// rows are not so aligned). Per-row statistics reduce over the TPR adjacent
// lanes of the row by shuffles. Versus conv_tile_epilogue: all waves store,
// NT/64 x fewer store instructions per byte, no register hand-over between
// waves. Output stride s_out == 1 only (the caller keeps conv_tile_epilogue
// for the stride-2 data-gradient phases).
// ---------------------------------------------------------------------------
constexpr int kEpiPitch = 260;  // floats: rows 4 words apart modulo 64 banks

template <int PITCH = kEpiPitch>
__device__ __forceinline__ void acc_to_img(float *img, const floatx16 &a, int row0, int col0) {
  const int lane = threadIdx.x & 63, hi = lane >> 5, lo = lane & 31;
#pragma unroll
  for (int i = 0; i < 16; ++i)
    img[(row0 + (i & 3) + 8 * (i >> 2) + 4 * hi) * PITCH + col0 + lo] = a[i];
}

// PF: every residual / bias-table load hoisted ahead of the stores (below);
// costs 4 PPT registers -- for one-workgroup-per-CU kernels only (at two per CU
// the extra registers halved the occupancy: +37% on the bf16 k_conv_x3)
template <int V, int NCOLS, int NT, int ROWS = 64, bool OB = false, bool PF = false>
__device__ __forceinline__ void conv_tile_store_rows(const ConvGemmParams &p, const float *img,
                                                     float *sbv, int n, int r0, int m0) {
  constexpr int TPR = NT / ROWS;
  static_assert(TPR >= 1 && NT % ROWS == 0, "whole threads per row");
  constexpr int NP = (NCOLS + 3) / 4;  // 16-byte pieces per row
  constexpr int PPT = (NP + TPR - 1) / TPR;
  const int tid = threadIdx.x;
  const int r = tid / TPR, q = tid - r * TPR;
  const int row = r0 + r;
  const bool rok = row < p.R;
  const int ostride = p.T_dst * V;
  const int ncv = min(NCOLS, (p.M - m0) * V);  // valid columns of the tile
  if (p.bias_rv) {  // the tile's rows of the bias table, coalesced (uniform branch)
    const int nrow = min(ROWS, p.R - r0);
    for (int i = tid; i < nrow * V; i += NT) sbv[i] = p.bias_rv[r0 * V + i];
    __syncthreads();
  }
  const float br = (p.bias_r && rok) ? p.bias_r[row] : 0.f;
  const int64_t obase = (int64_t)n * p.out_bstride + (int64_t)row * ostride + (int64_t)m0 * V;
  float *out = p.out + obase;
  // (res_shared: one table for every clip, so its offset has no clip term)
  const int64_t rbase = p.res_shared ? obase - (int64_t)n * p.out_bstride : obase;
  const float *res = p.res ? p.res + rbase : nullptr;
  const int vec = ((obase & 3) == 0 && (rbase & 3) == 0 && (ostride & 3) == 0 &&
                   ((reinterpret_cast<uintptr_t>(p.out) & 15) == 0) &&
                   (!p.res || (reinterpret_cast<uintptr_t>(p.res) & 15) == 0))
                      ? 4
                      : (((obase & 1) == 0 && (rbase & 1) == 0 && (ostride & 1) == 0) ? 2 : 1);
  double s = 0.0, sq = 0.0;
  // The residual / bias-table pieces, all loaded before the first store: vmcnt
  // counts stores and loads in one in-order counter, so a load issued after a
  // store can only be waited for together with that store -- loads interleaved
  // with the stores made every piece wait for the previous piece's store to
  // complete (its full write latency, PPT times per tile)
  float rq[PF ? PPT : 1][4];
#pragma unroll
  for (int k = 0; k < (PF ? PPT : 0); ++k) {
    const int pc = q + k * TPR, c0 = pc * 4;
#pragma unroll
    for (int e = 0; e < 4; ++e) rq[k][e] = 0.f;
    if (res && rok && pc < NP) {
      if (c0 + 3 < ncv && vec == 4) {
        const float4 t = *reinterpret_cast<const float4 *>(res + c0);
        rq[k][0] = t.x; rq[k][1] = t.y; rq[k][2] = t.z; rq[k][3] = t.w;
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e)
          if (c0 + e < ncv) rq[k][e] = res[c0 + e];
      }
    }
  }
#pragma unroll
  for (int k = 0; k < PPT; ++k) {
    const int pc = q + k * TPR;
    if (pc >= NP) break;
    const int c0 = pc * 4;
    const float4 a = *reinterpret_cast<const float4 *>(img + r * kEpiPitch + c0);
    float v[4] = {a.x, a.y, a.z, a.w};
    const bool full = rok && c0 + 3 < ncv;
    float rv[4] = {0.f, 0.f, 0.f, 0.f};
    if constexpr (PF) {
#pragma unroll
      for (int e = 0; e < 4; ++e) rv[e] = rq[k][e];
    } else if (res && rok) {
      if (full && vec == 4) {
        const float4 t = *reinterpret_cast<const float4 *>(res + c0);
        rv[0] = t.x; rv[1] = t.y; rv[2] = t.z; rv[3] = t.w;
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e)
          if (c0 + e < ncv) rv[e] = res[c0 + e];
      }
    }
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int col = c0 + e;
      const bool ok = rok && col < ncv;
      float val = v[e] + br;
      if (p.bias_rv && ok) val += sbv[r * V + col % V];
      val += rv[e];
      if (p.relu_out) val = fmaxf(val, 0.f);
      if (p.drop.thresh && ok)
        val = dropout_keep(p.drop, (uint64_t)(obase + col)) ? val * p.drop.scale : 0.f;
      v[e] = val;
      if (p.stat_sum && ok) {
        s += (double)val;
        sq += (double)val * (double)val;
      }
    }
    if (OB && p.out_bf16) {  // bf16 output: 8-byte pieces where the row allows
      __bf16 *ob = reinterpret_cast<__bf16 *>(p.out) + obase;
      const unsigned w0 = __builtin_bit_cast(unsigned short, (__bf16)v[0]) |
                          ((unsigned)__builtin_bit_cast(unsigned short, (__bf16)v[1]) << 16);
      const unsigned w1 = __builtin_bit_cast(unsigned short, (__bf16)v[2]) |
                          ((unsigned)__builtin_bit_cast(unsigned short, (__bf16)v[3]) << 16);
      if (full && vec == 4) {
        *reinterpret_cast<uint2 *>(ob + c0) = make_uint2(w0, w1);
      } else if (full && vec == 2) {
        *reinterpret_cast<unsigned *>(ob + c0) = w0;
        *reinterpret_cast<unsigned *>(ob + c0 + 2) = w1;
      } else if (rok) {
#pragma unroll
        for (int e = 0; e < 4; ++e)
          if (c0 + e < ncv) ob[c0 + e] = (__bf16)v[e];
      }
    } else if (full && vec == 4) {
      *reinterpret_cast<float4 *>(out + c0) = make_float4(v[0], v[1], v[2], v[3]);
    } else if (full && vec == 2) {
      *reinterpret_cast<float2 *>(out + c0) = make_float2(v[0], v[1]);
      *reinterpret_cast<float2 *>(out + c0 + 2) = make_float2(v[2], v[3]);
    } else if (rok) {
#pragma unroll
      for (int e = 0; e < 4; ++e)
        if (c0 + e < ncv) out[c0 + e] = v[e];
    }
  }
  if (p.stat_sum) {  // per-row sums over the TPR adjacent lanes of the row
#pragma unroll
    for (int o = 1; o < TPR; o <<= 1) {
      s += __shfl_xor(s, o, 64);
      sq += __shfl_xor(sq, o, 64);
    }
    if (p.stat_part) {  // (uniform) per-tile partials, plain stores
      if (q == 0 && rok) {
        const int64_t nt = (int64_t)p.N * p.n_mtiles;  // [2][R][tiles]: channel-major
        double *pt = p.stat_part + (int64_t)row * nt + (int64_t)n * p.n_mtiles + m0 / (NCOLS / V);
        pt[0] = s;
        pt[(int64_t)p.R * nt] = sq;
      }
    } else if (q == 0 && rok) {
      atomicAdd(p.stat_sum + row, s);
      atomicAdd(p.stat_sq + row, sq);
    }
  }
}

}  // namespace stgcn
