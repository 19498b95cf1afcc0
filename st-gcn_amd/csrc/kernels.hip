// Device code of libstgcn_hip.so — gfx950 (MI355X / CDNA4) only.
//
// GEMM-shaped work (the spatial 1x1 channel contraction, the (9,1) temporal
// convolution forward / data-grad / weight-grad) runs on the exact-fp32 matrix
// cores (v_mfma_f32_32x32x2_f32: one fmaf chain per output, no reduced
// precision). The joint-axis (V) contractions with the dense adjacency A run
// on the VALU from LDS (A pinned in LDS per workgroup). BatchNorm statistics
// accumulate in fp64.
//
// Wave size is 64; every block is a multiple of 64 threads.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <initializer_list>
#include <type_traits>

#include "device_common.h"
#include "internal.h"

namespace stgcn {


// ---------------------------------------------------------------------------
// conv_gemm: see ConvGemmParams. Workgroup = 256 threads (4 waves), tile =
// 64 rows x (FT frames * V) columns (<= 256, padded to 8 MFMA column tiles).
// Wave w owns rows (w&1)*32..+31 and column tiles (w>>1)*4..+3: 4 accumulators
// of 32x32 fp32 (64 VGPRs). The reduction runs over input-channel chunks of CK:
// each chunk's weights (pre-packed [rtile][c][q][64], a contiguous block) and
// input windows (frames + temporal halo, zero-padded) are staged global ->
// registers -> LDS, double-buffered: the loads of chunk i+1 are in flight while
// chunk i runs on the matrix cores; one barrier per chunk. Each staged channel
// window serves all NQ taps (the tap shift is a per-lane LDS offset).
// ---------------------------------------------------------------------------
// Packs w[r*w_sr + c*w_sc + q*w_sq] into wpk[rt][c][q][r_local] (zero padded
// to n_rtiles*64 rows and Cpad channels).
__global__ void k_pack_conv_w(const float *w, float *wpk, int R, int C, int Cpad, int NQ,
                              int64_t w_sr, int64_t w_sc, int64_t w_sq, int n_rtiles) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t total = (int64_t)n_rtiles * Cpad * NQ * 64;
  if (idx >= total) return;
  const int rl = (int)(idx & 63);
  int64_t t = idx >> 6;
  const int q = (int)(t % NQ);
  t /= NQ;
  const int c = (int)(t % Cpad);
  const int rt = (int)(t / Cpad);
  const int r = rt * 64 + rl;
  float v = 0.f;
  if (r < R && c < C) v = w[(int64_t)r * w_sr + (int64_t)c * w_sc + (int64_t)q * w_sq];
  wpk[idx] = v;
}

template <int NQ, int CK>
__global__ __launch_bounds__(256, 2) void k_conv_gemm(ConvGemmParams p) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  constexpr int WSZ = CK * NQ * 64;   // floats of one weight chunk (multiple of 256)
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int hi = lane >> 5, lo = lane & 31;
  const int nblk = gridDim.x;
  int bid = xcd_remap(blockIdx.x, nblk);
  const int rt = bid % p.n_rtiles;
  bid /= p.n_rtiles;
  const int mt = bid % p.n_mtiles;
  const int n = bid / p.n_mtiles;
  const int r0 = rt * kTileRows, m0 = mt * p.FT;
  const int V = p.V;
  const int span = (p.s_in * (p.FT - 1) + NQ) * V;
  const int SP = span | 1;  // odd pitch
  const int ISZ = round64(CK * SP);
  float *Ws0 = smem, *Ws1 = smem + WSZ;
  float *Is0 = smem + 2 * WSZ, *Is1 = smem + 2 * WSZ + ISZ;
  const int cstride = p.T_src * V;
  const int g0 = (p.s_in * m0 + p.off) * V;
  const float *inN = p.in + (int64_t)n * p.in_bstride;
  const float *wblk = p.wpk + (int64_t)rt * p.Cpad * NQ * 64;
  const int ncols = p.FT * V;
  const int nchunks = (p.C + CK - 1) / CK;

  const int mi = wave & 1;
  const int nj0 = (wave >> 1) * 4;
  int bbase[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int col = (nj0 + j) * 32 + lo;
    if (col < ncols) {
      const int mf = col / V;
      bbase[j] = p.s_in * mf * V + (col - mf * V);
    } else {
      bbase[j] = 0;  // padding column: reads a staged value, result discarded
    }
  }
  // LDS-DMA staging of chunk `chunk` into (Ws, Is). Input image [CK][SP]:
  // element e -> (c = e / SP, o = e % SP); this lane starts at e = wave*64+lane
  // and advances by 256 per instruction.
  const int e_init = wave * 64 + lane;
  const int c_init = e_init / SP, o_init = e_init - c_init * SP;
  const int dc = 256 / SP, dO = 256 - dc * SP;
  const __amdgpu_buffer_rsrc_t rs_w = make_rsrc(wblk, (int64_t)p.Cpad * NQ * 64);
  const __amdgpu_buffer_rsrc_t rs_in = make_rsrc(inN, (int64_t)p.C * cstride);
  auto stage = [&](int chunk, float *Ws, float *Is) {
    const unsigned wbase = (unsigned)(chunk * WSZ + wave * 64 + lane) * 4u;
#pragma unroll
    for (int i = 0; i < WSZ / 256; ++i) blds_f32(rs_w, wbase + i * 1024u, Ws + (i * 4 + wave) * 64);
    const int climit = p.C - chunk * CK;
    const int cbase = chunk * CK * cstride + g0;
    int c = c_init, o = o_init;
    for (int E0 = wave * 64; E0 < ISZ; E0 += 256) {
      const int g = g0 + o;
      const bool ok = c < CK && c < climit && o < span && g >= 0 && g < cstride;
      blds_f32(rs_in, ok ? (unsigned)(cbase + c * cstride + o) * 4u : kOOB, Is + E0);
      o += dO;
      c += dc;
      if (o >= SP) {
        o -= SP;
        ++c;
      }
    }
  };

  floatx16 acc[4];
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[j][i] = 0.f;

  stage(0, Ws0, Is0);
  __syncthreads();
  for (int chunk = 0; chunk < nchunks; ++chunk) {
    const bool odd = chunk & 1;
    const float *Ws = odd ? Ws1 : Ws0;
    const float *Is = odd ? Is1 : Is0;
    if (chunk + 1 < nchunks) stage(chunk + 1, odd ? Ws0 : Ws1, odd ? Is0 : Is1);
    const float *wp = Ws + hi * NQ * 64 + mi * 32 + lo;
    const float *ip = Is + hi * SP;
#pragma unroll 2
    for (int cp = 0; cp < CK / 2; ++cp) {
#pragma unroll
      for (int q = 0; q < NQ; ++q) {
        const float a = wp[(2 * cp * NQ + q) * 64];
        const float *iq = ip + 2 * cp * SP + q * V;
        const float b0 = iq[bbase[0]], b1 = iq[bbase[1]], b2 = iq[bbase[2]], b3 = iq[bbase[3]];
        acc[0] = mfma32(a, b0, acc[0]);
        acc[1] = mfma32(a, b1, acc[1]);
        acc[2] = mfma32(a, b2, acc[2]);
        acc[3] = mfma32(a, b3, acc[3]);
      }
    }
    __syncthreads();  // retires this wave's LDS-DMA (vmcnt(0)) and publishes the next chunk
  }

  // Epilogue: bias, store, optional per-row BN statistics (fp64).
  float *outN = p.out + (int64_t)n * p.out_bstride;
  const int64_t ostride = (int64_t)p.T_dst * V;
  int64_t ocol[4];
  bool cok[4];
  int cv[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int col = (nj0 + j) * 32 + lo;
    const int mf = col / V;
    const int v = col - mf * V;
    const int m = m0 + mf;
    cok[j] = col < ncols && m < p.M;
    cv[j] = v;
    ocol[j] = (int64_t)(p.s_out * m + p.p_out) * V + v;
  }
  // per-lane partial BN statistics (fp64 over this lane's 4 columns), summed
  // across lanes and waves through LDS (the staging buffers are free now).
  double *red = reinterpret_cast<double *>(smem);  // [4 waves][16 regs][2][64 lanes]
  // (every load ahead of the stores that follow it: vmcnt counts loads and
  // stores in one in-order counter, so a load issued after a store is only
  // waited for together with that store. Row biases first; bias-table and
  // residual values one register ahead of their stores)
  float brv[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const int row = r0 + mi * 32 + (i & 3) + 8 * (i >> 2) + 4 * hi;
    brv[i] = (row < p.R && p.bias_r) ? p.bias_r[row] : 0.f;
  }
  const float *resN = p.res ? p.res + (p.res_shared ? 0 : (int64_t)n * p.out_bstride) : nullptr;
  float pbv[2][4], prs[2][4];
  auto pre = [&](int i, float (&bv)[4], float (&rs)[4]) {
    const int row = r0 + mi * 32 + (i & 3) + 8 * (i >> 2) + 4 * hi;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      bv[j] = 0.f;
      rs[j] = 0.f;
      if (row < p.R && cok[j]) {
        if (p.bias_rv) bv[j] = p.bias_rv[row * V + cv[j]];
        if (resN) rs[j] = resN[row * ostride + ocol[j]];
      }
    }
  };
  pre(0, pbv[0], prs[0]);
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    if (i + 1 < 16) pre(i + 1, pbv[(i + 1) & 1], prs[(i + 1) & 1]);
    const int row = r0 + mi * 32 + (i & 3) + 8 * (i >> 2) + 4 * hi;
    const bool rok = row < p.R;
    const float br = brv[i];
    double s = 0.0, sq = 0.0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      if (rok && cok[j]) {
        float val = acc[j][i] + br;
        if (p.bias_rv) val += pbv[i & 1][j];
        if (p.res) val += prs[i & 1][j];
        if (p.relu_out) val = fmaxf(val, 0.f);
        if (p.drop.thresh)
          val = dropout_keep(p.drop, (uint64_t)n * p.out_bstride + row * ostride + ocol[j])
                    ? val * p.drop.scale
                    : 0.f;
        outN[row * ostride + ocol[j]] = val;
        s += val;
        sq += (double)val * val;
      }
    }
    if (p.stat_sum) {
      red[((wave * 16 + i) * 2 + 0) * 64 + lane] = s;
      red[((wave * 16 + i) * 2 + 1) * 64 + lane] = sq;
    }
  }
  if (p.stat_sum) {
    __syncthreads();
    if (tid < 128) {
      // row rl of the tile: wave halves mi = rl / 32 (waves mi and mi + 2),
      // register i and lane half h from rl % 32 = (i&3) + 8*(i>>2) + 4*h
      const int rl = tid >> 1, st = tid & 1;
      const int m = rl >> 5, rr = rl & 31;
      const int h = (rr >> 2) & 1, i = (rr & 3) + 4 * (rr >> 3);
      double acc_s = 0.0;
      for (int w = m; w < 4; w += 2) {
        const double *src = red + ((w * 16 + i) * 2 + st) * 64 + h * 32;
        // rotated start: the 32 lanes of a wave half read 32 different banks
        for (int l = 0; l < 32; ++l) acc_s += src[(l + tid) & 31];
      }
      const int row = r0 + rl;
      if (row < p.R) atomicAdd((st ? p.stat_sq : p.stat_sum) + row, acc_s);
    }
  }
}

// ---------------------------------------------------------------------------
// k_tconv: conv_gemm specialised on the joint count V and the input stride
// (FT = kTileCols / V frames per tile). With the image geometry known at
// compile time every LDS operand read is (per-lane base + immediate), the
// input DMA offsets of a lane are the same for every channel chunk (computed
// once; the chunk and the channel bound live in the buffer resource, so the
// last partial chunk and the temporal halo zero-fill through the hardware
// range check), the packed-weight chunk moves in 16-byte LDS-DMA pieces, and
// the k-loop is fully unrolled with explicitly double-buffered operands (the
// LDS reads of step s+1 are in flight under the 4 MFMAs of step s).
// ---------------------------------------------------------------------------
template <int NQ, int CK, int V, int SIN>
struct ConvGeo {
  static constexpr int FT = kTileCols / V;
  static constexpr int NCOLS = FT * V;
  static constexpr int SPAN = (SIN * (FT - 1) + NQ) * V;
  static constexpr int SP = SPAN | 1;  // odd pitch
  static constexpr int ISZ = round64(CK * SP);
  static constexpr int WSZ = CK * NQ * 64;
  static constexpr int IROWS = ISZ / 64;              // 64-float DMA rows of the input image
  static constexpr int NI = (IROWS + 3) / 4;          // rows per wave (upper bound)
  static constexpr int WROWS = (WSZ + 255) / 256;     // 256-float (16 B/lane) weight rows
  static constexpr int WLAST = (WSZ % 256) / 4;       // lanes of a partial last row (0: full)
  static constexpr int NS = CK / 2 * NQ;              // MFMA k-steps per chunk
  static_assert(CK % 2 == 0 && WSZ % 4 == 0, "k-steps pair channels; 16-byte weight pieces");
  // ring-buffered staging: the chunk's DMA rows (WROWS 16-byte weight rows,
  // then input rows) are dealt round-robin to the 4 waves, padded with extra
  // input rows (zero-filled, never read) so every wave issues DPW DMAs.
  static constexpr int DPW = (WROWS + IROWS + 3) / 4;   // DMAs per wave per chunk
  static constexpr int IROWS_P = 4 * DPW - WROWS;       // input rows incl. padding
  static constexpr int WBUF = WROWS * 256, IBUF = IROWS_P * 64;
  static constexpr int BUF = WBUF + IBUF;               // floats per ring slot
  // ring depth: 3 slots (the short spatial chunks too: 2 slots measured 4-5%
  // slower at the cfg2 layer shapes once bias_rv moved to LDS)
#ifndef STGCN_STAGES1
#define STGCN_STAGES1 3
#endif
  static constexpr int STAGES = NQ == 1 ? STGCN_STAGES1 : 3;
  static_assert((STAGES - 2) * DPW < 64, "vmcnt range");
  // Input stride 2: each channel's window is stored de-interleaved, even
  // frames first (NFE of them) then odd frames, so output column (mf, v) at
  // tap q reads position TAPOFF(q) + mf*V + v: consecutive columns hit
  // consecutive words (the interleaved layout read 2- to 3-way bank conflicts).
  static constexpr int NF = SPAN / V;                  // window frames
  static constexpr int NFE = (NF + 1) / 2;             // even frames
  static __host__ __device__ constexpr int tapoff(int q) {
    return SIN == 2 ? (q & 1) * NFE * V + (q >> 1) * V : q * V;
  }
  // window position (de-interleaved layout) -> frame offset within the window
  static __host__ __device__ constexpr int src_pos(int o) {
    return SIN != 2 ? o
                    : (o < NFE * V ? 2 * (o / V) * V + o % V
                                   : (2 * ((o - NFE * V) / V) + 1) * V + (o - NFE * V) % V);
  }
};

template <int NQ, int CK, int V, int SIN>
__global__ __launch_bounds__(256, 2) void k_tconv(ConvGemmParams p) {
  using G = ConvGeo<NQ, CK, V, SIN>;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int hi = lane >> 5, lo = lane & 31;
  int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int rt = bid % p.n_rtiles;
  bid /= p.n_rtiles;
  const int mt = bid % p.n_mtiles;
  const int n = bid / p.n_mtiles;
  const int r0 = rt * kTileRows, m0 = mt * G::FT;
  const int cstride = p.T_src * V;
  const int g0 = (SIN * m0 + p.off) * V;
  const float *inN = p.in + (int64_t)n * p.in_bstride;
  const float *wblk = p.wpk + (int64_t)rt * p.Cpad * NQ * 64;
  const int nchunks = (p.C + CK - 1) / CK;
  const int mi = wave & 1;
  const int nj0 = (wave >> 1) * 4;

  int bb[4];  // per-lane LDS offset of this lane's B column (k-row hi) in the image
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int col = (nj0 + j) * 32 + lo;
    const int mf = col / V;
    bb[j] = hi * G::SP + (col < G::NCOLS ? (SIN == 2 ? col : SIN * mf * V + (col - mf * V)) : 0);
  }
  // DMA slot k of this wave: row d = 4k + wave; d < WROWS: weight row d
  // (16 B/lane), else input row d - WROWS (4 B/lane, byte offset voff[k]
  // relative to the chunk's first channel; kOOB outside the image)
  unsigned voff[G::DPW];
#pragma unroll
  for (int k = 0; k < G::DPW; ++k) {
    const int d = 4 * k + wave;
    const int e = (d - G::WROWS) * 64 + lane;
    const int c = e / G::SP, o = e - c * G::SP;
    const int g = g0 + (o < G::SPAN ? G::src_pos(o) : o);
    const bool ok = d >= G::WROWS && c < CK && o < G::SPAN && g >= 0 && g < cstride;
    voff[k] = ok ? (unsigned)(c * cstride + g) * 4u : kOOB;
  }
  const __amdgpu_buffer_rsrc_t rs_w = make_rsrc(wblk, (int64_t)p.Cpad * NQ * 64);
  auto stage = [&](int chunk, float *Ws, float *Is) {
    const __amdgpu_buffer_rsrc_t rs_in =
        make_rsrc(inN + (int64_t)chunk * CK * cstride, (int64_t)(p.C - chunk * CK) * cstride);
#pragma unroll
    for (int k = 0; k < G::DPW; ++k) {
      const int d = 4 * k + wave;  // wave-uniform
      if (d < G::WROWS) {
        // a partial last weight row still issues (OOB lanes: zero) so that every
        // wave's DMA count stays DPW
        const bool lane_ok = G::WLAST == 0 || d < G::WROWS - 1 || lane < G::WLAST;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(
            rs_w, Ws + d * 256, 16,
            lane_ok ? (unsigned)(chunk * G::WSZ + d * 256 + lane * 4) * 4u : kOOB, 0, 0, 0);
      } else {
        blds_f32(rs_in, voff[k], Is + (d - G::WROWS) * 64);
      }
    }
  };

  floatx16 acc[4];
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[j][i] = 0.f;

  // STAGES-slot ring: chunks c+1 .. c+STAGES-1 are in flight while chunk c
  // computes. Each wave waits only for its own DMAs of chunk c (vmcnt counts
  // retire in order), then one barrier publishes the chunk (a fenced
  // __syncthreads would drain the whole ring).
  constexpr int S = G::STAGES;
  auto wbuf = [&](int slot) { return smem + slot * G::BUF; };
  auto ibuf = [&](int slot) { return smem + slot * G::BUF + G::WBUF; };
#pragma unroll
  for (int c = 0; c < S - 1; ++c)
    if (c < nchunks) stage(c, wbuf(c), ibuf(c));
  auto body = [&](int chunk, auto slot_c) {
    constexpr int SLOT = decltype(slot_c)::value;
    if (S == 3 && chunk + 1 < nchunks)  // chunk c+1 may stay in flight
      asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" ::"n"((S - 2) * G::DPW) : "memory");
    else
      asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
    if (chunk + S - 1 < nchunks)
      stage(chunk + S - 1, wbuf((SLOT + S - 1) % S), ibuf((SLOT + S - 1) % S));
    const float *Ws = wbuf(SLOT), *Is = ibuf(SLOT);
    const float *wp = Ws + hi * NQ * 64 + mi * 32 + lo;
    const float *ib0 = Is + bb[0], *ib1 = Is + bb[1], *ib2 = Is + bb[2], *ib3 = Is + bb[3];
    constexpr int PD = 2;  // operands are read PD k-steps ahead of their MFMAs
    float a[PD + 1], b[PD + 1][4];
    auto ld = [&](int s, int set) {
      const int cp = s / NQ, q = s - cp * NQ;
      const int bo = 2 * cp * G::SP + G::tapoff(q);
      a[set] = wp[(2 * cp * NQ + q) * 64];
      b[set][0] = ib0[bo];
      b[set][1] = ib1[bo];
      b[set][2] = ib2[bo];
      b[set][3] = ib3[bo];
    };
#pragma unroll
    for (int s = 0; s < PD && s < G::NS; ++s) ld(s, s);
#pragma unroll
    for (int s = 0; s < G::NS; ++s) {
      if (s + PD < G::NS) ld(s + PD, (s + PD) % (PD + 1));
      const int c = s % (PD + 1);
      acc[0] = mfma32(a[c], b[c][0], acc[0]);
      acc[1] = mfma32(a[c], b[c][1], acc[1]);
      acc[2] = mfma32(a[c], b[c][2], acc[2]);
      acc[3] = mfma32(a[c], b[c][3], acc[3]);
      // issue order per step: step s+PD's 5 LDS reads, then step s's 4 MFMAs
      __builtin_amdgcn_sched_group_barrier(0x100, 5, 0);
      __builtin_amdgcn_sched_group_barrier(0x008, 4, 0);
      __builtin_amdgcn_sched_barrier(0);
    }
  };
  static_assert(S == 2 || S == 3, "ring depth");
  for (int chunk = 0; chunk < nchunks; chunk += S) {
    body(chunk, std::integral_constant<int, 0>{});
    if (chunk + 1 < nchunks) body(chunk + 1, std::integral_constant<int, 1>{});
    if constexpr (S == 3)
      if (chunk + 2 < nchunks) body(chunk + 2, std::integral_constant<int, 2 % S>{});
  }
  asm volatile("s_barrier" ::: "memory");  // every wave done reading the ring (LDS reuse)

  conv_tile_epilogue<V, G::NCOLS, NQ == 1>(p, acc, n, r0, m0, smem);
}




// The (V, stride, NQ) combinations with a specialised k_tconv instantiation:
// the joint counts of the reference's skeleton graphs (coco18, body25,
// two-person body25), input stride 1 (and 2 for the strided temporal forward).
static bool tconv_specialised(const ConvGemmParams &p) {
  if (STGCN_AB_GENERIC_CONV) return false;  // A/B builds only (ab_switches.h)
  if (p.V != 18 && p.V != 25 && p.V != 50) return false;
  if (p.FT != kTileCols / p.V) return false;
  if (p.s_in == 2) return p.NQ == 9;
  return p.s_in == 1 && (p.NQ == 1 || p.NQ == 4 || p.NQ == 5 || p.NQ == 9);
}

// Channels per reduction chunk. Specialised kernels: 8 for the spatial GEMM
// (2-slot ring), 2 for the temporal taps (3-slot ring, 27 KB of LDS: 4
// workgroups per CU); measured against 16/32 and 4/6/8 (scripts/ck_sweep.sh).
#ifndef STGCN_CK1
#define STGCN_CK1 8
#endif
#ifndef STGCN_CK45
#define STGCN_CK45 2
#endif
static int conv_ck(const ConvGemmParams &p) {
  if (!tconv_specialised(p)) return p.NQ == 1 ? 32 : 8;
  return p.NQ == 1 ? STGCN_CK1 : (p.NQ == 4 || p.NQ == 5) ? STGCN_CK45 : 2;
}

int conv_gemm_cpad(const ConvGemmParams &p) {
  const int CK = conv_ck(p);
  return (p.C + CK - 1) / CK * CK;
}

size_t conv_gemm_wpk_floats(const ConvGemmParams &p) {
  return (size_t)p.n_rtiles * conv_gemm_cpad(p) * p.NQ * 64;
}

int conv_gemm_span(const ConvGemmParams &p) { return (p.s_in * (p.FT - 1) + p.NQ) * p.V; }

size_t conv_gemm_lds_bytes(const ConvGemmParams &p) {
  const int CK = conv_ck(p);
  const size_t stage = sizeof(float) * 2 * ((size_t)CK * p.NQ * 64 + round64(CK * (conv_gemm_span(p) | 1)));
  if (tconv_specialised(p)) {  // ring of ConvGeo::STAGES slots; stats partials (2 KiB) reuse it
    const int WROWS = (CK * p.NQ * 64 + 255) / 256;
    const int IROWS = round64(CK * (conv_gemm_span(p) | 1)) / 64;
    const int DPW = (WROWS + IROWS + 3) / 4;
    const int stages = p.NQ == 1 ? STGCN_STAGES1 : 3;
    return sizeof(float) * stages * ((size_t)WROWS * 256 + (size_t)(4 * DPW - WROWS) * 64);
  }
  const size_t stats = sizeof(double) * 4 * 16 * 2 * 64;  // k_conv_gemm epilogue buffer
  return stage > stats ? stage : stats;
}

bool conv_gemm_supported(const ConvGemmParams &p) {
  return p.FT * p.V <= kTileCols && conv_gemm_lds_bytes(p) <= 160 * 1024;
}

template <int NQ, int CK, int V, int SIN>
static bool launch_tconv_if(const ConvGemmParams &p, int nblk, size_t lds, hipStream_t s) {
  if (p.V != V || p.s_in != SIN || p.FT != ConvGeo<NQ, CK, V, SIN>::FT) return false;
  hipLaunchKernelGGL((k_tconv<NQ, CK, V, SIN>), dim3(nblk), dim3(256), lds, s, p);
  return true;
}

template <int NQ, int CK>
static bool launch_tconv_v(const ConvGemmParams &p, int nblk, size_t lds, hipStream_t s) {
  if (launch_tconv_if<NQ, CK, 18, 1>(p, nblk, lds, s)) return true;
  if (launch_tconv_if<NQ, CK, 25, 1>(p, nblk, lds, s)) return true;
  if (launch_tconv_if<NQ, CK, 50, 1>(p, nblk, lds, s)) return true;
  if constexpr (NQ == 9) {
    if (launch_tconv_if<NQ, CK, 18, 2>(p, nblk, lds, s)) return true;
    if (launch_tconv_if<NQ, CK, 25, 2>(p, nblk, lds, s)) return true;
    if (launch_tconv_if<NQ, CK, 50, 2>(p, nblk, lds, s)) return true;
  }
  return false;
}

template <int NQ>
static bool launch_tconv_ck(const ConvGemmParams &p, int CK, int nblk, size_t lds,
                            hipStream_t s) {
  if constexpr (NQ == 1) {
    if (CK == STGCN_CK1) return launch_tconv_v<NQ, STGCN_CK1>(p, nblk, lds, s);
  } else if constexpr (NQ == 4 || NQ == 5) {
    if (CK == STGCN_CK45) return launch_tconv_v<NQ, STGCN_CK45>(p, nblk, lds, s);
  } else {
    if (CK == 2) return launch_tconv_v<NQ, 2>(p, nblk, lds, s);
  }
  return false;
}

hipError_t launch_conv_gemm(const ConvGemmParams &p0, hipStream_t s) {
  // (per-tile statistics partials: k_conv_x3's row-major epilogue only)
  if (p0.stat_part && (p0.s_out != 1 || !p0.stat_sum)) return hipErrorInvalidValue;
  if (p0.bf16 == 3 && conv_x3_supported(p0)) return launch_conv_x3(p0, s);
  // (the fused SpatialConv backward epilogue and the fp16 operand scales exist in
  // k_conv_x3 only: any other kernel would ignore them and write H / wrong results)
  if (p0.spb || p0.f16x2 || p0.stat_part) return hipErrorInvalidValue;
  if (p0.bf16 == 1 && conv_b1_supported(p0)) return launch_conv_b1(p0, s);
  if (p0.bf16 == 1 && conv_bf16_supported(p0)) return launch_conv_bf16(p0, s);
  // (bf16-stored operands: only the kernels above read / write them)
  if (p0.in_bf16 || p0.out_bf16) return hipErrorInvalidValue;
  ConvGemmParams p = p0;
  if (!conv_gemm_supported(p) || !p.wpk) return hipErrorInvalidValue;
  p.Cpad = conv_gemm_cpad(p);
  {
    const int64_t total = (int64_t)conv_gemm_wpk_floats(p);
    hipLaunchKernelGGL(k_pack_conv_w, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s,
                       p.w, p.wpk, p.R, p.C, p.Cpad, p.NQ, p.w_sr, p.w_sc, p.w_sq, p.n_rtiles);
  }
  const int nblk = p.N * p.n_mtiles * p.n_rtiles;
  const size_t lds = conv_gemm_lds_bytes(p);
  if (tconv_specialised(p)) {
    const int CK = conv_ck(p);
    bool done = false;
    switch (p.NQ) {
      case 1:
        done = launch_tconv_ck<1>(p, CK, nblk, lds, s);
        break;
      case 4:
        done = launch_tconv_ck<4>(p, CK, nblk, lds, s);
        break;
      case 5:
        done = launch_tconv_ck<5>(p, CK, nblk, lds, s);
        break;
      case 9:
        done = launch_tconv_ck<9>(p, CK, nblk, lds, s);
        break;
    }
    return done ? hipGetLastError() : hipErrorInvalidValue;
  }
  switch (p.NQ) {
    case 1:
      hipLaunchKernelGGL((k_conv_gemm<1, 32>), dim3(nblk), dim3(256), lds, s, p);
      break;
    case 4:
      hipLaunchKernelGGL((k_conv_gemm<4, 8>), dim3(nblk), dim3(256), lds, s, p);
      break;
    case 5:
      hipLaunchKernelGGL((k_conv_gemm<5, 8>), dim3(nblk), dim3(256), lds, s, p);
      break;
    case 9:
      hipLaunchKernelGGL((k_conv_gemm<9, 8>), dim3(nblk), dim3(256), lds, s, p);
      break;
    default:
      return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// wgrad: see WgradParams. Workgroup = 256 threads, output tile 64 rows (r) x
// JT columns (j = c*NQ + q), JT = 192 (NQ=9) or 128 (NQ=1). Wave w owns rows
// (w&1)*32..+31 and column tiles (w>>1)*NJW..+NJW-1 (NJW = JT/64). The
// reduction runs over work items (clip n, FT frames): P[64 rows][FT*V cols]
// and the Q channel windows of the tile's j range are staged global ->
// registers -> LDS, double-buffered; one barrier per item. The split's partial
// tile is written to its slab (reduced in fixed order by k_slab_reduce).
// ---------------------------------------------------------------------------
template <int NQ, int JT>
__global__ __launch_bounds__(256, 2) void k_wgrad(WgradParams p) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  constexpr int NJW = JT / 64;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int hi = lane >> 5, lo = lane & 31;
  const int nblk = gridDim.x;
  int bid = xcd_remap(blockIdx.x, nblk);
  const int split = bid % p.S;
  bid /= p.S;
  const int jt = bid % p.n_jtiles;
  const int rt = bid / p.n_jtiles;
  const int r0 = rt * 64, j0 = jt * JT;
  const int J = p.C * NQ;
  const int V = p.V;
  const int Vp = (V + 1) & ~1;          // joints padded to even: k-steps never straddle frames
  const int ncols = p.FT * Vp;          // P image columns (frame-padded)
  const int PP = ncols | 1;             // odd pitch
  const int c_lo = j0 / NQ;
  int c_hi = (j0 + JT - 1) / NQ + 1;
  if (c_hi > p.C) c_hi = p.C;
  const int nc = c_hi - c_lo;
  const int span = (p.s_in * (p.FT - 1) + NQ) * V;
  const int QP = (span + 2) | 1;        // >= span + 1: the odd-V pad column reads a finite value
  const int PSZ = round64(64 * PP), QSZ = round64((nc + 1) * QP);  // Q row nc = zeros
  float *Ps0 = smem, *Qs0 = smem + PSZ;
  float *Ps1 = smem + PSZ + QSZ, *Qs1 = Ps1 + PSZ;
  const int mi = wave & 1;
  const int nj0 = (wave >> 1) * NJW;
  int qoff[NJW];
#pragma unroll
  for (int t = 0; t < NJW; ++t) {
    const int j = j0 + (nj0 + t) * 32 + lo;
    if (j < J) {
      const int c = j / NQ, q = j - c * NQ;
      qoff[t] = (c - c_lo) * QP + q * V;
    } else {
      qoff[t] = nc * QP;  // zero row
    }
  }
  floatx16 acc[NJW];
#pragma unroll
  for (int t = 0; t < NJW; ++t)
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[t][i] = 0.f;

  const int total = p.N * p.n_mtiles;
  const int per = (total + p.S - 1) / p.S;
  const int it0 = split * per;
  int it1 = it0 + per;
  if (it1 > total) it1 = total;
  const int pcs = p.M * V;      // P channel stride
  const int qcs = p.T_src * V;  // Q channel stride
  // per-lane staging walk: element e = wave*64 + lane + 256*i of each image
  const int e_init = wave * 64 + lane;
  const int prow_i = e_init / PP, po_i = e_init - prow_i * PP;
  const int dpr = 256 / PP, dpo = 256 - dpr * PP;
  const int qrow_i = e_init / QP, qo_i = e_init - qrow_i * QP;
  const int dqr = 256 / QP, dqo = 256 - dqr * QP;
  const int prow_lim = min(64, p.R - r0);

  // LDS-DMA staging of work item `it`: P image [64][PP] (frame-padded columns)
  // and Q image [nc+1][QP]; out-of-range elements read as 0 (buffer OOB).
  auto stage = [&](int it, float *Ps, float *Qs) {
    const int n = it / p.n_mtiles, mt = it - n * p.n_mtiles;
    const int m0 = mt * p.FT;
    const __amdgpu_buffer_rsrc_t rs_p =
        make_rsrc(p.P + (int64_t)n * p.p_bstride + (int64_t)r0 * pcs, (int64_t)prow_lim * pcs);
    const int fl = p.M - m0;  // frames left in this clip
    int row = prow_i, o = po_i;
    for (int E0 = wave * 64; E0 < PSZ; E0 += 256) {
      const int mf = o / Vp, v = o - mf * Vp;
      const bool ok = row < prow_lim && o < ncols && v < V && mf < fl;
      blds_f32(rs_p, ok ? (unsigned)(row * pcs + (m0 + mf) * V + v) * 4u : kOOB, Ps + E0);
      o += dpo;
      row += dpr;
      if (o >= PP) {
        o -= PP;
        ++row;
      }
    }
    const int qg0 = (p.s_in * m0 + p.off) * V;
    const __amdgpu_buffer_rsrc_t rs_q =
        make_rsrc(p.Q + (int64_t)n * p.q_bstride + (int64_t)c_lo * qcs, (int64_t)nc * qcs);
    row = qrow_i;
    o = qo_i;
    for (int E0 = wave * 64; E0 < QSZ; E0 += 256) {
      const int g = qg0 + o;
      const bool ok = row < nc && o < span && g >= 0 && g < qcs;
      blds_f32(rs_q, ok ? (unsigned)(row * qcs + g) * 4u : kOOB, Qs + E0);
      o += dqo;
      row += dqr;
      if (o >= QP) {
        o -= QP;
        ++row;
      }
    }
  };

  const int hv = Vp / 2;  // k-steps per frame
  if (it0 < it1) stage(it0, Ps0, Qs0);
  __syncthreads();
  for (int it = it0; it < it1; ++it) {
    const bool odd = (it - it0) & 1;
    const float *Ps = odd ? Ps1 : Ps0;
    const float *Qs = odd ? Qs1 : Qs0;
    if (it + 1 < it1) stage(it + 1, odd ? Ps0 : Ps1, odd ? Qs0 : Qs1);
    // k-steps walk the frame-padded P columns contiguously (A offset += 2) and
    // the Q window of each frame (B offset += 2, jump s*V - Vp per frame).
    // Operands of step k+1 are read before the MFMAs of step k.
    const float *pa = Ps + (mi * 32 + lo) * PP + hi;
    const float *qb = Qs + hi;
    const int nsteps = p.FT * hv;
    const int fjump = p.s_in * V - Vp;
    int aoff = 0, boff = 0, kin = 0;
    float a_cur = pa[0];
    float b_cur[NJW];
#pragma unroll
    for (int t = 0; t < NJW; ++t) b_cur[t] = qb[qoff[t]];
    for (int kk = 0; kk < nsteps - 1; ++kk) {
      aoff += 2;
      boff += 2;
      if (++kin == hv) {
        kin = 0;
        boff += fjump;
      }
      const float a_nxt = pa[aoff];
      float b_nxt[NJW];
#pragma unroll
      for (int t = 0; t < NJW; ++t) b_nxt[t] = qb[qoff[t] + boff];
#pragma unroll
      for (int t = 0; t < NJW; ++t) acc[t] = mfma32(a_cur, b_cur[t], acc[t]);
      a_cur = a_nxt;
#pragma unroll
      for (int t = 0; t < NJW; ++t) b_cur[t] = b_nxt[t];
    }
#pragma unroll
    for (int t = 0; t < NJW; ++t) acc[t] = mfma32(a_cur, b_cur[t], acc[t]);
    __syncthreads();  // retires this wave's LDS-DMA and publishes the next item
  }
  float *dst = p.slab + (int64_t)split * p.R * J;
#pragma unroll
  for (int t = 0; t < NJW; ++t)
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int row = r0 + mi * 32 + (i & 3) + 8 * (i >> 2) + 4 * hi;
      const int j = j0 + (nj0 + t) * 32 + lo;
      if (row < p.R && j < J) dst[(int64_t)row * J + j] = acc[t][i];
    }
}

// ---------------------------------------------------------------------------
// wgrad_taps: the (9,1) temporal conv weight gradient,
//   dWt[r][c][q] = sum_{n,m,v} P[n,r,m,v] * Q[n,c, s*m + q + off, v],
// tile = 64 rows x CB channels x all 9 taps. 4 waves; wave w: rows
// (w&1)*32..+31; CB=64: channels (w>>1)*32..+31, taps 0..8 (9 MFMA tiles);
// CB=32: all 32 channels, taps (w>>1) ? 5..8 : 0..4. MFMA column tiles are
// tap-major/channel-minor, so a B read is 32 lanes on 32 channel rows of an
// odd-pitch image (conflict-free) and one A read feeds up to 9 MFMAs.
// Work items (clip n, FT frames) are staged by LDS-DMA, double-buffered.
// ---------------------------------------------------------------------------
// VT > 0: specialised on the joint count VT, input stride SIN and FTT frames
// per item (compile-time image geometry, fully unrolled scheduled k-loop);
// VT = 0: runtime geometry.
template <int CB, int NW, int VT, int SIN, int FTT>
__global__ __launch_bounds__(NW * 64, 1) void k_wgrad_taps(WgradParams p) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  // waves: (row half mi, channel half cb, tap group qh); CB=64/NW=8 -> 2x2x2,
  // CB=32/NW=4 -> 2x1x2; tap groups 0..4 and 5..8
  constexpr int NT = 5;  // MFMA column tiles per wave
  constexpr int NTH = NW * 64;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int hi = lane >> 5, lo = lane & 31;
  const int nblk = gridDim.x;
  int bid = xcd_remap(blockIdx.x, nblk);
  const int split = bid % p.S;
  bid /= p.S;
  const int ct = bid % p.n_jtiles;
  const int rt = bid / p.n_jtiles;
  const int r0 = rt * 64, c0 = ct * CB;
  const int V = VT ? VT : p.V;
  const int FT = VT ? FTT : p.FT;
  const int s_in = VT ? SIN : p.s_in;
  const int Vp = (V + 1) & ~1;
  const int ncols = FT * Vp;
  const int PP = ncols | 1;
  const int span = (s_in * (FT - 1) + 9) * V;
  const int QP = (span + 2) | 1;
  // images padded to whole DMA rounds of the workgroup (every wave issues the
  // same number of DMAs; the padding reads as zero)
  const int PSZ = (64 * PP + NTH - 1) / NTH * NTH, QSZ = (CB * QP + NTH - 1) / NTH * NTH;
  float *Ps0 = smem, *Qs0 = smem + PSZ;
  float *Ps1 = smem + PSZ + QSZ, *Qs1 = Ps1 + PSZ;
  const int mi = wave & 1;
  const int cb = CB == 64 ? ((wave >> 1) & 1) : 0;
  const int qh = CB == 64 ? (wave >> 2) : (wave >> 1);
  const int q0 = qh ? 5 : 0;
  const int nq = qh ? 4 : 5;
  int qoff[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) qoff[t] = (cb * 32 + lo) * QP + (q0 + t) * V;
  floatx16 acc[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[t][i] = 0.f;

  const int total = p.N * p.n_mtiles;
  const int per = (total + p.S - 1) / p.S;
  const int it0 = split * per;
  int it1 = it0 + per;
  if (it1 > total) it1 = total;
  const int pcs = p.M * V;
  const int qcs = p.T_src * V;
  const int prow_lim = min(64, p.R - r0);
  const int crow_lim = min(CB, p.C - c0);
  // P staging: per-lane element list is the same for every item; precompute
  // packed (offset | frame << 26), -1 when statically out of range.
  constexpr int MAXPE = VT ? (64 * ((FTT * ((VT + 1) & ~1)) | 1) + NTH - 1) / NTH
                          : 24 * 4 / NW;  // >= ceil(64 * PP / NTH) for PP <= 95
  int ppk[MAXPE];
  const int npe = PSZ / NTH;
  {
#pragma unroll
    for (int i = 0; i < MAXPE; ++i) {
      const int e = (i * NW + wave) * 64 + lane;
      const int row = e / PP, o = e - row * PP;
      const int mf = o / Vp, v = o - mf * Vp;
      const bool ok = i < npe && row < prow_lim && o < ncols && v < V;
      ppk[i] = ok ? ((row * pcs + mf * V + v) | (mf << 26)) : -1;
    }
  }
  const int qrow_i = (wave * 64 + lane) / QP, qo_i = (wave * 64 + lane) - qrow_i * QP;
  const int dqr = NTH / QP, dqo = NTH - dqr * QP;
  // Specialised geometry: the Q element list of a lane is also fixed per item;
  // precompute packed (row*qcs + o) | (o << 21), -1 when statically out of range
  // (qcs * 64 < 2^21 and o < 2^10 for the instantiated V, T <= 300).
  constexpr int QN = VT ? (CB * ((((SIN * (FTT - 1) + 9) * VT) + 2) | 1) + NTH - 1) / NTH : 1;
  int qpk[QN];
  if constexpr (VT > 0) {
#pragma unroll
    for (int i = 0; i < QN; ++i) {
      const int e = (i * NW + wave) * 64 + lane;
      const int row = e / QP, o = e - row * QP;
      const bool ok = row < crow_lim && o < span;
      qpk[i] = ok ? ((row * qcs + o) | (o << 21)) : -1;
    }
  }

  auto stage = [&](int it, float *Ps, float *Qs) {
    const int n = it / p.n_mtiles, mt = it - n * p.n_mtiles;
    const int m0 = mt * FT;
    const int fl = p.M - m0;
    const __amdgpu_buffer_rsrc_t rs_p =
        make_rsrc(p.P + (int64_t)n * p.p_bstride + (int64_t)r0 * pcs, (int64_t)prow_lim * pcs);
    const int m0V = m0 * V;
#pragma unroll
    for (int i = 0; i < MAXPE; ++i) {
      if (VT > 0 || i < npe) {
        const int pk = ppk[i];
        const bool ok = pk >= 0 && (pk >> 26) < fl;
        blds_f32(rs_p, ok ? (unsigned)((pk & 0x3ffffff) + m0V) * 4u : kOOB,
                 Ps + (i * NW + wave) * 64);
      }
    }
    const int qg0 = (s_in * m0 + p.off) * V;
    const __amdgpu_buffer_rsrc_t rs_q =
        make_rsrc(p.Q + (int64_t)n * p.q_bstride + (int64_t)c0 * qcs, (int64_t)crow_lim * qcs);
    if constexpr (VT > 0) {
      // interior items (no temporal halo outside the clip) skip the frame test
      auto qdma = [&](auto interior_c) {
        constexpr bool INTERIOR = decltype(interior_c)::value;
#pragma unroll
        for (int i = 0; i < QN; ++i) {
          const int pk = qpk[i];
          bool ok = pk >= 0;
          if constexpr (!INTERIOR) {
            const int g = qg0 + (pk >> 21);
            ok = ok && g >= 0 && g < qcs;
          }
          blds_f32(rs_q, ok ? (unsigned)((pk & 0x1fffff) + qg0) * 4u : kOOB,
                   Qs + (i * NW + wave) * 64);
        }
      };
      if (qg0 >= 0 && qg0 + span <= qcs)
        qdma(std::true_type{});
      else
        qdma(std::false_type{});
      return;
    }
    int row = qrow_i, o = qo_i;
    for (int E0 = wave * 64; E0 < QSZ; E0 += NTH) {
      const int g = qg0 + o;
      const bool ok = row < crow_lim && o < span && g >= 0 && g < qcs;
      blds_f32(rs_q, ok ? (unsigned)(row * qcs + g) * 4u : kOOB, Qs + E0);
      o += dqo;
      row += dqr;
      if (o >= QP) {
        o -= QP;
        ++row;
      }
    }
  };

  const int hv = Vp / 2;
  const int nsteps = FT * hv;
  const int fjump = s_in * V - Vp;
  if (it0 < it1) stage(it0, Ps0, Qs0);
  __syncthreads();
  for (int it = it0; it < it1; ++it) {
    const bool odd = (it - it0) & 1;
    const float *Ps = odd ? Ps1 : Ps0;
    const float *Qs = odd ? Qs1 : Qs0;
    if (it + 1 < it1) stage(it + 1, odd ? Ps0 : Ps1, odd ? Qs0 : Qs1);
    const float *pa = Ps + (mi * 32 + lo) * PP + hi;
    const float *qb = Qs + hi;
    if constexpr (VT > 0) {
      // fully unrolled; issue order per step: step k+PD's reads, then step k's MFMAs
      constexpr int HV = ((VT + 1) & ~1) / 2, NS = FTT * HV;
      constexpr int FJ = SIN * VT - 2 * HV;
      const float *qb0 = qb + qoff[0], *qb1 = qb + qoff[1], *qb2 = qb + qoff[2];
      const float *qb3 = qb + qoff[3], *qb4 = qb + qoff[4];
      const float *qbt[NT] = {qb0, qb1, qb2, qb3, qb4};
      // the tap count of the wave (5 or 4) is a template constant of the loop
      // body; operands are read PD steps ahead of their MFMAs (PD + 1 sets)
      auto body = [&](auto nqc) {
        constexpr int NQW = decltype(nqc)::value;
        constexpr int PD = 2;
        float a[PD + 1], b[PD + 1][NQW];
        auto ld = [&](int k, int set) {
          const int bo = 2 * k + (k / HV) * FJ;
          a[set] = pa[2 * k];
#pragma unroll
          for (int t = 0; t < NQW; ++t) b[set][t] = qbt[t][bo];
        };
#pragma unroll
        for (int k = 0; k < PD; ++k) ld(k, k);
#pragma unroll
        for (int k = 0; k < NS; ++k) {
          if (k + PD < NS) ld(k + PD, (k + PD) % (PD + 1));
          const int c = k % (PD + 1);
#pragma unroll
          for (int t = 0; t < NQW; ++t) acc[t] = mfma32(a[c], b[c][t], acc[t]);
          __builtin_amdgcn_sched_group_barrier(0x100, NQW + 1, 0);
          __builtin_amdgcn_sched_group_barrier(0x008, NQW, 0);
          __builtin_amdgcn_sched_barrier(0);
        }
      };
      if (qh)
        body(std::integral_constant<int, 4>{});
      else
        body(std::integral_constant<int, 5>{});
      __syncthreads();
      continue;
    }
    // 2x-unrolled ping-pong operand sets: the reads of step k+1 are issued
    // before the MFMAs of step k and land in the other register set (no
    // rotation moves, so the wait before step k+1 covers only its own reads).
    int aoff = 0, boff = 0, kin = 0;
    auto advance = [&]() {
      aoff += 2;
      boff += 2;
      if (++kin == hv) {
        kin = 0;
        boff += fjump;
      }
    };
    float a0 = pa[0], a1 = 0.f;
    float b0[NT], b1[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t) b0[t] = qb[qoff[t]];
    int kk = 0;
    for (; kk + 1 < nsteps; kk += 2) {
      advance();
      a1 = pa[aoff];
#pragma unroll
      for (int t = 0; t < NT; ++t) b1[t] = qb[qoff[t] + boff];
#pragma unroll
      for (int t = 0; t < NT; ++t)
        if (t < nq) acc[t] = mfma32(a0, b0[t], acc[t]);
      if (kk + 2 < nsteps) {
        advance();
        a0 = pa[aoff];
#pragma unroll
        for (int t = 0; t < NT; ++t) b0[t] = qb[qoff[t] + boff];
      }
#pragma unroll
      for (int t = 0; t < NT; ++t)
        if (t < nq) acc[t] = mfma32(a1, b1[t], acc[t]);
    }
    if (kk < nsteps) {
#pragma unroll
      for (int t = 0; t < NT; ++t)
        if (t < nq) acc[t] = mfma32(a0, b0[t], acc[t]);
    }
    __syncthreads();  // retires this wave's LDS-DMA and publishes the next item
  }
  // slab layout = the Conv2d weight (R, C, 9)
  float *dst = p.slab + (int64_t)split * p.R * p.C * 9;
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    if (t >= nq) continue;
    const int c = c0 + cb * 32 + lo;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int row = r0 + mi * 32 + (i & 3) + 8 * (i >> 2) + 4 * hi;
      if (row < p.R && c < p.C) dst[((int64_t)row * p.C + c) * 9 + q0 + t] = acc[t][i];
    }
  }
}

int wgrad_taps_cb(const WgradParams &p) { return p.V > 32 ? 32 : 64; }

size_t wgrad_taps_lds_bytes(const WgradParams &p) {
  const int CB = wgrad_taps_cb(p);
  const int NTH = CB == 64 ? 512 : 256;
  const int Vp = (p.V + 1) & ~1;
  const int PP = (p.FT * Vp) | 1;
  const int QP = ((p.s_in * (p.FT - 1) + 9) * p.V + 2) | 1;
  auto rnd = [&](int x) { return (x + NTH - 1) / NTH * NTH; };
  return sizeof(float) * 2 * (rnd(64 * PP) + rnd(CB * QP));
}

bool wgrad_taps_supported(const WgradParams &p) {
  const int Vp = (p.V + 1) & ~1;
  const int PP = (p.FT * Vp) | 1;
  return p.NQ == 9 && (64 * PP + 255) / 256 <= 24 && wgrad_taps_lds_bytes(p) <= 160 * 1024;
}

hipError_t launch_wgrad_taps(const WgradParams &p, hipStream_t s) {
  if (p.bf16 == 3) return launch_wgrad_x3(p, s);
  if (p.bf16) return launch_wgrad_bf16(p, s);
  if (!wgrad_taps_supported(p)) return hipErrorInvalidValue;
  const int nblk = p.n_rtiles * p.n_jtiles * p.S;
  const size_t lds = wgrad_taps_lds_bytes(p);
  if (!STGCN_AB_GENERIC_CONV) {
    // the plans make_wgrad_taps builds for the reference's graphs (FT = 80 / V,
    // reduced until the double-buffered images fit in LDS)
    if (p.V == 18 && p.FT == 4 && p.s_in == 1)
      hipLaunchKernelGGL((k_wgrad_taps<64, 8, 18, 1, 4>), dim3(nblk), dim3(512), lds, s, p);
    else if (p.V == 18 && p.FT == 3 && p.s_in == 2)
      hipLaunchKernelGGL((k_wgrad_taps<64, 8, 18, 2, 3>), dim3(nblk), dim3(512), lds, s, p);
    else if (p.V == 25 && p.FT == 2 && p.s_in == 1)
      hipLaunchKernelGGL((k_wgrad_taps<64, 8, 25, 1, 2>), dim3(nblk), dim3(512), lds, s, p);
    else if (p.V == 25 && p.FT == 1 && p.s_in == 2)
      hipLaunchKernelGGL((k_wgrad_taps<64, 8, 25, 2, 1>), dim3(nblk), dim3(512), lds, s, p);
    else if (p.V == 50 && p.FT == 1 && p.s_in == 1)
      hipLaunchKernelGGL((k_wgrad_taps<32, 4, 50, 1, 1>), dim3(nblk), dim3(256), lds, s, p);
    else if (p.V == 50 && p.FT == 1 && p.s_in == 2)
      hipLaunchKernelGGL((k_wgrad_taps<32, 4, 50, 2, 1>), dim3(nblk), dim3(256), lds, s, p);
    else
      goto generic_path;
    return hipGetLastError();
  }
generic_path:
  if (wgrad_taps_cb(p) == 64)
    hipLaunchKernelGGL((k_wgrad_taps<64, 8, 0, 1, 1>), dim3(nblk), dim3(512), lds, s, p);
  else
    hipLaunchKernelGGL((k_wgrad_taps<32, 4, 0, 1, 1>), dim3(nblk), dim3(256), lds, s, p);
  return hipGetLastError();
}

static int wgrad_jt(int NQ) { return NQ == 1 ? 128 : 192; }

static void wgrad_geom(const WgradParams &p, int &PP, int &nc, int &QP) {
  const int JT = wgrad_jt(p.NQ);
  PP = (p.FT * ((p.V + 1) & ~1)) | 1;
  nc = JT / p.NQ + 2;
  if (nc > p.C) nc = p.C;
  QP = ((p.s_in * (p.FT - 1) + p.NQ) * p.V + 2) | 1;
}

int wgrad_ntiles_j(int C, int NQ) { return (C * NQ + wgrad_jt(NQ) - 1) / wgrad_jt(NQ); }

size_t wgrad_lds_bytes(const WgradParams &p) {
  int PP, nc, QP;
  wgrad_geom(p, PP, nc, QP);
  return sizeof(float) * 2 * (round64(64 * PP) + round64((nc + 1) * QP));
}

bool wgrad_supported(const WgradParams &p) { return wgrad_lds_bytes(p) <= 160 * 1024; }

// ---------------------------------------------------------------------------
// k_wgrad_sp: weight gradient of the 1x1 spatial conv (NQ = 1) as a split-K GEMM
//   slab[split][r][c] = sum_{(n, chunk) in split} sum_{l in chunk} P[n][r][l] Q[n][c][l]
// over the L = T*V contiguous columns of each clip row, in chunks of KC. Both
// operands are staged row-major [rows][PITCH = KC + 4] (PITCH/4 odd: each
// 16-lane group of a ds_read_b128 hits 16 distinct 16-byte slots), by 16-byte
// LDS-DMA when rows are 16-byte aligned, else 4-byte. One ds_read_b128 per
// operand feeds 4 MFMAs: lane (i, h) holds k = kb + 4h + u for MFMA u, the same
// k permutation on both operands. Workgroups of one split are consecutive in
// the (XCD-remapped) grid, so the tiles sharing a chunk share an L2.
// X3 (STGCN_F_F32X3 blocks): the same staging, the products as exact 3-way bf16
// splits on v_mfma_f32_32x32x16_bf16 (six products, h*h apart; kernels_x3.hip):
// 16-deep k-steps, lane half h holding k = kb + 8h + u (u < 8) of both operands
// (two 16-byte reads per operand), split in registers at fragment read.
// ---------------------------------------------------------------------------
typedef __bf16 wsp_bf8 __attribute__((ext_vector_type(8)));
typedef __bf16 wsp_bf2 __attribute__((ext_vector_type(2)));
typedef float wsp_f4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ unsigned wsp_pk(float a, float b) {
  const wsp_bf2 v = {(__bf16)a, (__bf16)b};
  return __builtin_bit_cast(unsigned, v);
}
// 8 floats (two 16-byte LDS reads) -> exact bf16 planes h, m, l (x == h + m + l)
__device__ __forceinline__ void wsp_planes(const float *src, uint4 &h, uint4 &m, uint4 &l) {
  const wsp_f4 *v = reinterpret_cast<const wsp_f4 *>(__builtin_assume_aligned(src, 16));
  const wsp_f4 x0 = v[0], x1 = v[1];
  const float f[8] = {x0.x, x0.y, x0.z, x0.w, x1.x, x1.y, x1.z, x1.w};
  unsigned hh[4], mm[4], ll[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const float a = f[2 * i], b = f[2 * i + 1];
    hh[i] = wsp_pk(a, b);
    const float ra = a - __builtin_bit_cast(float, hh[i] << 16);
    const float rb = b - __builtin_bit_cast(float, hh[i] & 0xffff0000u);
    mm[i] = wsp_pk(ra, rb);
    ll[i] = wsp_pk(ra - __builtin_bit_cast(float, mm[i] << 16),
                   rb - __builtin_bit_cast(float, mm[i] & 0xffff0000u));
  }
  h = uint4{hh[0], hh[1], hh[2], hh[3]};
  m = uint4{mm[0], mm[1], mm[2], mm[3]};
  l = uint4{ll[0], ll[1], ll[2], ll[3]};
}
__device__ __forceinline__ floatx16 wsp_mfma(uint4 a, uint4 b, floatx16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(wsp_bf8, a),
                                                 __builtin_bit_cast(wsp_bf8, b), c, 0, 0, 0);
}

// NS > 2 (X3 only): an NS-slot LDS-DMA ring with hand-counted waits (items
// it+1 .. it+NS-2 in flight while item it computes; one workgroup per CU).
template <int CT, bool X4>
struct WspGeo {
  static constexpr int KC = CT == 64 ? 64 : 32, PITCH = KC + 4;
  static constexpr int PSZ = 64 * PITCH, QSZ = CT * PITCH;
  static constexpr int G = X4 ? 4 : 1;
  // DMA wave-instructions per item; every wave issues at least DMIN of them
  static constexpr int NPW = (PSZ / G + 63) / 64, NQW = (QSZ / G + 63) / 64;
  static constexpr int DMIN = NPW / 4 + NQW / 4;
  static constexpr int RING = 2 * DMIN < 64 ? 4 : 3;  // vmcnt allowance (NS-2)*DMIN < 64
};

template <int CT, bool X4, bool X3, int NS = 2>
__global__ __launch_bounds__(256, 2) void k_wgrad_sp(WgradParams p) {
  constexpr int KC = CT == 64 ? 64 : 32, PITCH = KC + 4;
  static_assert((PITCH / 4) % 2 == 1, "ds_read_b128 conflict-free pitch");
  constexpr int PSZ = 64 * PITCH, QSZ = CT * PITCH;
  constexpr int NJ = CT / 64;               // 32-column accumulators per wave
  constexpr int G = X4 ? 4 : 1;             // floats per lane per DMA
  constexpr int PN = (PSZ / G + 255) / 256;  // DMA rounds per wave (upper bound)
  constexpr int QN = (QSZ / G + 255) / 256;
  static_assert(NS == 2 || (X3 && NS <= WspGeo<CT, X4>::RING), "ring only on the x3 path");
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float *Ps0 = smem, *Qs0 = smem + PSZ, *Ps1 = smem + PSZ + QSZ, *Qs1 = Ps1 + PSZ;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int hi = lane >> 5, lo = lane & 31;
  int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int ntiles = p.n_rtiles * p.n_jtiles;
  const int tile = bid % ntiles;
  const int split = bid / ntiles;
  const int ct = tile % p.n_jtiles, rt = tile / p.n_jtiles;
  const int L = p.M * p.V;
  const int r0 = rt * 64, c0 = ct * CT;
  const int prow_lim = min(64, p.R - r0), qrow_lim = min(CT, p.C - c0);
  const int total = p.N * p.n_mtiles;
  const int per = (total + p.S - 1) / p.S;
  const int it0 = split * per;
  const int it1 = min(total, it0 + per);

  // fixed per-lane staging map: DMA round i of this wave fills LDS floats
  // [((i*4 + wave)*64 + lane) * G, +G) of the image
  int poff[PN], pcol[PN], qoff[QN], qcol[QN];
#pragma unroll
  for (int i = 0; i < PN; ++i) {
    const int pos = ((i * 4 + wave) * 64 + lane) * G;
    const int row = pos / PITCH, col = pos - row * PITCH;
    pcol[i] = col;
    poff[i] = (pos < PSZ && col < KC && row < prow_lim) ? row * L + col : -1;
  }
#pragma unroll
  for (int i = 0; i < QN; ++i) {
    const int pos = ((i * 4 + wave) * 64 + lane) * G;
    const int row = pos / PITCH, col = pos - row * PITCH;
    qcol[i] = col;
    qoff[i] = (pos < QSZ && col < KC && row < qrow_lim) ? row * L + col : -1;
  }
  auto dma = [&](__amdgpu_buffer_rsrc_t rs, unsigned voff, float *lds) {
    if constexpr (X4)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, lds, 16, voff, 0, 0, 0);
    else
      blds_f32(rs, voff, lds);
  };
  auto stage = [&](int it, float *Ps, float *Qs) {
    const int n = it / p.n_mtiles, kc = it - n * p.n_mtiles;
    const int l0 = kc * KC, lrem = L - l0;
    const __amdgpu_buffer_rsrc_t rs_p = make_rsrc(
        p.P + (int64_t)n * p.p_bstride + (int64_t)r0 * L + l0, (int64_t)prow_lim * L - l0);
    const __amdgpu_buffer_rsrc_t rs_q = make_rsrc(
        p.Q + (int64_t)n * p.q_bstride + (int64_t)c0 * L + l0, (int64_t)qrow_lim * L - l0);
#pragma unroll
    for (int i = 0; i < PN; ++i) {
      if ((i * 4 + wave) * 64 * G < PSZ) {
        const bool ok = poff[i] >= 0 && pcol[i] < lrem;
        dma(rs_p, ok ? (unsigned)poff[i] * 4u : kOOB, Ps + (i * 4 + wave) * 64 * G);
      }
    }
#pragma unroll
    for (int i = 0; i < QN; ++i) {
      if ((i * 4 + wave) * 64 * G < QSZ) {
        const bool ok = qoff[i] >= 0 && qcol[i] < lrem;
        dma(rs_q, ok ? (unsigned)qoff[i] * 4u : kOOB, Qs + (i * 4 + wave) * 64 * G);
      }
    }
  };

  const int mi = wave & 1, nj = wave >> 1;
  floatx16 acc[NJ], acl[NJ];
#pragma unroll
  for (int t = 0; t < NJ; ++t)
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[t][i] = acl[t][i] = 0.f;
  // x3 products of one staged item (P rows at Ps, Q rows at Qs)
  auto x3_item = [&](const float *Ps, const float *Qs) {
    const float *pa = Ps + (mi * 32 + lo) * PITCH + 8 * hi;
    const float *qb = Qs + (nj * (CT / 2) + lo) * PITCH + 8 * hi;
#pragma unroll
    for (int s = 0; s < KC / 16; ++s) {
      uint4 ah, am, al, bh[NJ], bm[NJ], bl[NJ];
      wsp_planes(pa + 16 * s, ah, am, al);
#pragma unroll
      for (int t = 0; t < NJ; ++t) wsp_planes(qb + t * 32 * PITCH + 16 * s, bh[t], bm[t], bl[t]);
#pragma unroll
      for (int t = 0; t < NJ; ++t) {
        acc[t] = wsp_mfma(ah, bh[t], acc[t]);
        acl[t] = wsp_mfma(ah, bm[t], acl[t]);
        acl[t] = wsp_mfma(am, bh[t], acl[t]);
        acl[t] = wsp_mfma(ah, bl[t], acl[t]);
        acl[t] = wsp_mfma(am, bm[t], acl[t]);
        acl[t] = wsp_mfma(al, bh[t], acl[t]);
      }
    }
  };
  if constexpr (NS > 2) {
    constexpr int D = WspGeo<CT, X4>::DMIN, SLOT = PSZ + QSZ;
#pragma unroll
    for (int k = 0; k < NS - 1; ++k)
      if (it0 + k < it1) stage(it0 + k, smem + k * SLOT, smem + k * SLOT + PSZ);
    int sl = 0;
    for (int it = it0; it < it1; ++it) {
      const int ahead = min(NS - 2, it1 - 1 - it);  // items staged after this one
      if (ahead >= 2)
        asm volatile("s_waitcnt vmcnt(%0)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::"n"(2 * D) : "memory");
      else if (ahead == 1)
        asm volatile("s_waitcnt vmcnt(%0)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::"n"(D) : "memory");
      else
        asm volatile("s_waitcnt vmcnt(0)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
      if (it + NS - 1 < it1) {
        float *nx = smem + (sl == 0 ? NS - 1 : sl - 1) * SLOT;
        stage(it + NS - 1, nx, nx + PSZ);
      }
      x3_item(smem + sl * SLOT, smem + sl * SLOT + PSZ);
      sl = sl + 1 == NS ? 0 : sl + 1;
    }
  } else {
  if (it0 < it1) stage(it0, Ps0, Qs0);
  __syncthreads();
  for (int it = it0; it < it1; ++it) {
    const bool odd = (it - it0) & 1;
    const float *Ps = odd ? Ps1 : Ps0;
    const float *Qs = odd ? Qs1 : Qs0;
    if (it + 1 < it1) stage(it + 1, odd ? Ps0 : Ps1, odd ? Qs0 : Qs1);
    if constexpr (X3) {
      x3_item(Ps, Qs);
      __syncthreads();  // retires this wave's LDS-DMA and publishes the next chunk
      continue;
    }
    const float *pa = Ps + (mi * 32 + lo) * PITCH + 4 * hi;
    const float *qb = Qs + (nj * (CT / 2) + lo) * PITCH + 4 * hi;
    // element-wise reads (merged into ds_read_b128 by the backend; a float4
    // load here loses the alias info that keeps the next chunk's LDS-DMA from
    // being waited on before these reads); k-block s+1 is read before the
    // MFMAs of k-block s.
    float a[2][4], b[2][NJ][4];
    auto ld = [&](int kb, int set) {
#pragma unroll
      for (int u = 0; u < 4; ++u) a[set][u] = pa[kb + u];
#pragma unroll
      for (int t = 0; t < NJ; ++t)
#pragma unroll
        for (int u = 0; u < 4; ++u) b[set][t][u] = qb[t * 32 * PITCH + kb + u];
    };
    ld(0, 0);
#pragma unroll
    for (int s = 0; s < KC / 8; ++s) {
      if (s + 1 < KC / 8) ld((s + 1) * 8, (s + 1) & 1);
      const int c = s & 1;
#pragma unroll
      for (int t = 0; t < NJ; ++t)
#pragma unroll
        for (int u = 0; u < 4; ++u) acc[t] = mfma32(a[c][u], b[c][t][u], acc[t]);
      __builtin_amdgcn_sched_group_barrier(0x100, 1 + NJ, 0);
      __builtin_amdgcn_sched_group_barrier(0x008, 4 * NJ, 0);
      __builtin_amdgcn_sched_barrier(0);
    }
    __syncthreads();  // retires this wave's LDS-DMA and publishes the next chunk
  }
  }
  float *dst = p.slab + (int64_t)split * p.R * p.C;
#pragma unroll
  for (int t = 0; t < NJ; ++t) {
    const int c = c0 + nj * (CT / 2) + t * 32 + lo;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int row = r0 + mi * 32 + (i & 3) + 8 * (i >> 2) + 4 * hi;
      if (row < p.R && c < p.C) dst[(int64_t)row * p.C + c] = X3 ? acc[t][i] + acl[t][i] : acc[t][i];
    }
  }
}

void plan_wgrad_sp(WgradParams &w) {
  w.CT = w.C <= 64 ? 64 : 128;
  const int KC = wgrad_sp_kc(w.CT);
  const int L = w.M * w.V;
  w.n_mtiles = (L + KC - 1) / KC;
  w.n_rtiles = (w.R + 63) / 64;
  w.n_jtiles = (w.C + w.CT - 1) / w.CT;
  const int tiles = w.n_rtiles * w.n_jtiles;
  w.S = std::max(1, std::min((512 + tiles - 1) / tiles, w.N * w.n_mtiles));
}

static hipError_t launch_wgrad_sp(const WgradParams &p, hipStream_t s) {
  if ((p.CT != 64 && p.CT != 128) || p.n_mtiles != (p.M * p.V + wgrad_sp_kc(p.CT) - 1) /
                                                       wgrad_sp_kc(p.CT))
    return hipErrorInvalidValue;
  const int64_t L = (int64_t)p.M * p.V;
  const bool x4 = L % 4 == 0 && p.p_bstride % 4 == 0 && p.q_bstride % 4 == 0 &&
                  ((uintptr_t)p.P & 15) == 0 && ((uintptr_t)p.Q & 15) == 0;
  const int nblk = p.n_rtiles * p.n_jtiles * p.S;
  const int KC = wgrad_sp_kc(p.CT);
  const size_t lds = sizeof(float) * 2 * (size_t)(64 + p.CT) * (KC + 4);
  const bool x3 = p.bf16 == 3;
  // x3: STGCN_AB_WSP_RING builds select the LDS-DMA ring (WspGeo::RING slots, one
  // workgroup per CU): measured 1% SLOWER on cfg2 than the two-buffer schedule
  // at two workgroups per CU (4356-4375 vs 4403-4415 clips/s in one A/B call);
  // A/B measurement only
  constexpr bool ring = STGCN_AB_WSP_RING != 0;
#define WSP_LAUNCH(CT, X4, X3)                                                              \
  do {                                                                                      \
    constexpr int NSR = WspGeo<CT, X4>::RING;                                               \
    if (X3 && ring)                                                                         \
      hipLaunchKernelGGL((k_wgrad_sp<CT, X4, X3, X3 ? NSR : 2>), dim3(nblk), dim3(256),     \
                         sizeof(float) * NSR * (size_t)(64 + CT) * (WspGeo<CT, X4>::KC + 4), s, p); \
    else                                                                                    \
      hipLaunchKernelGGL((k_wgrad_sp<CT, X4, X3>), dim3(nblk), dim3(256), lds, s, p);       \
  } while (0)
  if (p.CT == 64) {
    if (x4)
      { if (x3) WSP_LAUNCH(64, true, true); else WSP_LAUNCH(64, true, false); }
    else
      { if (x3) WSP_LAUNCH(64, false, true); else WSP_LAUNCH(64, false, false); }
  } else {
    if (x4)
      { if (x3) WSP_LAUNCH(128, true, true); else WSP_LAUNCH(128, true, false); }
    else
      { if (x3) WSP_LAUNCH(128, false, true); else WSP_LAUNCH(128, false, false); }
  }
#undef WSP_LAUNCH
  return hipGetLastError();
}

bool wgrad_sp_applies(const WgradParams &p) {
  return p.NQ == 1 && p.s_in == 1 && p.off == 0 && p.M == p.T_src;
}

hipError_t launch_wgrad(const WgradParams &p, hipStream_t s) {
  if (p.bf16 == 3 && wgrad_sp_applies(p)) return launch_wgrad_sp(p, s);  // x3 products
  if (p.bf16) return launch_wgrad_bf16(p, s);
  if (wgrad_sp_applies(p)) return launch_wgrad_sp(p, s);
  if (!wgrad_supported(p)) return hipErrorInvalidValue;
  const int nblk = p.n_rtiles * p.n_jtiles * p.S;
  const size_t lds = wgrad_lds_bytes(p);
  switch (p.NQ) {
    case 1:  // strided 1x1 (residual projection)
      hipLaunchKernelGGL((k_wgrad<1, 128>), dim3(nblk), dim3(256), lds, s, p);
      break;
    case 9:
      hipLaunchKernelGGL((k_wgrad<9, 192>), dim3(nblk), dim3(256), lds, s, p);
      break;
    default:
      return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

// Block = 32 consecutive outputs x 8 split groups (group g sums splits
// g, g+8, ... in fp64); the 8 partials are combined in a fixed order, so the
// result is deterministic.
__global__ __launch_bounds__(256) void k_slab_reduce(const float *slab, int S, int64_t n,
                                                     float *dst, int mode, int R, int K, int C) {
  __shared__ double red[8][33];
  const int o = threadIdx.x & 31, g = threadIdx.x >> 5;
  const int64_t idx = (int64_t)blockIdx.x * 32 + o;
  double s = 0.0;
  if (idx < n) {
#pragma unroll 8
    for (int k = g; k < S; k += 8) s += slab[(int64_t)k * n + idx];
  }
  red[g][o] = s;
  __syncthreads();
  if (g != 0 || idx >= n) return;
#pragma unroll
  for (int j = 1; j < 8; ++j) s += red[j][o];
  int64_t d = idx;
  if (mode == 1) {  // idx = co*(K*C) + k*C + ci  ->  (k*R + co)*C + ci
    const int64_t KC = (int64_t)K * C;
    const int64_t co = idx / KC, rem = idx - co * KC;
    const int64_t k = rem / C, ci = rem - k * C;
    d = (k * R + co) * C + ci;
  }
  dst[d] = (float)s;
}

hipError_t launch_slab_reduce(const float *slab, int S, int64_t n, float *dst, int mode, int R,
                              int K, int C, hipStream_t s) {
  const int nb = (int)((n + 31) / 32);
  hipLaunchKernelGGL(k_slab_reduce, dim3(nb), dim3(256), 0, s, slab, S, n, dst, mode, R, K, C);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// BatchNorm kernels. One 256-thread block per (n, c) slice of L = T*V floats.
// ---------------------------------------------------------------------------
// Vector width VEC (1, 2, 4 floats) for the per-(n, c) slice loops: the slice
// base (n*C + c)*L is a multiple of VEC when L is.
template <int N>
struct VecF;
template <>
struct VecF<1> {
  using T = float;
};
template <>
struct VecF<2> {
  using T = float2;
};
template <>
struct VecF<4> {
  using T = float4;
};
template <int N>
__device__ __forceinline__ void vld(const float *p, float (&v)[N]) {
  const typename VecF<N>::T t = *reinterpret_cast<const typename VecF<N>::T *>(p);
  __builtin_memcpy(v, &t, sizeof(t));
}
template <int N>
__device__ __forceinline__ void vst(float *p, const float (&v)[N]) {
  typename VecF<N>::T t;
  __builtin_memcpy(&t, v, sizeof(t));
  *reinterpret_cast<typename VecF<N>::T *>(p) = t;
}

static int slice_vec(int L, std::initializer_list<const void *> ptrs) {
  int vec = L % 4 == 0 ? 4 : (L % 2 == 0 ? 2 : 1);
  for (const void *q : ptrs)  // (null pointers are aligned)
    while (vec > 1 && ((uintptr_t)q & (4 * vec - 1)) != 0) vec >>= 1;
  return vec;
}

#define STGCN_VEC_LAUNCH(kern, vec, grid, ...)                            \
  do {                                                                    \
    if ((vec) == 4)                                                       \
      hipLaunchKernelGGL((kern<4>), grid, dim3(256), 0, s, __VA_ARGS__); \
    else if ((vec) == 2)                                                  \
      hipLaunchKernelGGL((kern<2>), grid, dim3(256), 0, s, __VA_ARGS__); \
    else                                                                  \
      hipLaunchKernelGGL((kern<1>), grid, dim3(256), 0, s, __VA_ARGS__); \
  } while (0)

// (amax, or null: max |x| as float bits, device_common.h block_amax -- the
// fp16 operand bound of the folded block's GEMMs that read x, capi.hip fold_bna)
template <int VEC>
__global__ __launch_bounds__(256) void k_bn_stats(const float *x, int C, int L, double *sum,
                                                  double *sq, unsigned *amax) {
  __shared__ double red[8];
  const int c = blockIdx.x, n = blockIdx.y;
  const float *src = x + ((int64_t)n * C + c) * L;
  double s = 0.0, q = 0.0;
  float m = 0.f;
  for (int i = threadIdx.x * VEC; i < L; i += 256 * VEC) {
    float v[VEC];
    vld<VEC>(src + i, v);
#pragma unroll
    for (int j = 0; j < VEC; ++j) {
      s += (double)v[j];
      q += (double)v[j] * (double)v[j];
      m = fmaxf(m, fabsf(v[j]));
    }
  }
  if (amax) block_amax<256>(m, amax);
  block_sum2_atomic<256>(s, q, sum + c, sq + c, red);
}

hipError_t launch_bn_stats(const float *x, int N, int C, int L, double *sum, double *sq,
                           hipStream_t s, unsigned *amax) {
  STGCN_VEC_LAUNCH(k_bn_stats, slice_vec(L, {x}), dim3(C, N), x, C, L, sum, sq, amax);
  return hipGetLastError();
}

// (zw non-null: also zeroes nzw words for the kernels that follow -- the f16x2
// max |x| words of the folded forward -- instead of a memset launch)
__global__ void k_bn_finalize(const double *sum, const double *sq, int C, int64_t M, float eps,
                              float momentum, int training, float *rm, float *rv, float *mean_out,
                              float *invstd_out, unsigned *zw, int nzw) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (zw)
    for (int i = c; i < nzw; i += gridDim.x * blockDim.x) zw[i] = 0u;
  if (c >= C) return;
  if (training) {
    const double mean = sum[c] / (double)M;
    double var = sq[c] / (double)M - mean * mean;
    if (var < 0.0) var = 0.0;
    mean_out[c] = (float)mean;
    invstd_out[c] = (float)(1.0 / sqrt(var + (double)eps));
    if (rm) {
      const double unb = M > 1 ? var * (double)M / (double)(M - 1) : var;
      rm[c] = (float)((1.0 - momentum) * rm[c] + momentum * mean);
      rv[c] = (float)((1.0 - momentum) * rv[c] + momentum * unb);
    }
  } else {
    mean_out[c] = rm[c];
    invstd_out[c] = (float)(1.0 / sqrt((double)rv[c] + (double)eps));
  }
}

// one workgroup per channel: the tile partials summed in a fixed order (strided
// per thread, then a fixed tree), then k_bn_finalize's arithmetic
// (ys non-null: also zeroes the block's y_stats -- 5 C doubles, then nw words --
// for the output pass that follows: no memset launch)
__global__ __launch_bounds__(256) void k_bn_finalize_parts(const double *part, int ntiles, int C,
                                                           int64_t M, float eps, float momentum,
                                                           int training, float *rm, float *rv,
                                                           float *mean_out, float *invstd_out,
                                                           double *ys, int nw) {
  __shared__ double red[2][256];
  const int c = blockIdx.x, tid = threadIdx.x;
  if (ys) {
    if (tid < 5) ys[(int64_t)tid * C + c] = 0.0;
    const int per = (nw + C - 1) / C;
    unsigned *w = reinterpret_cast<unsigned *>(ys + 5 * (int64_t)C);
    for (int i = tid; i < per; i += 256)
      if (c * per + i < nw) w[c * per + i] = 0u;
  }
  double a = 0.0, b = 0.0;
  const double *pa = part + (int64_t)c * ntiles, *pb = pa + (int64_t)C * ntiles;
  for (int t = tid; t < ntiles; t += 256) {  // (contiguous per channel: coalesced)
    a += pa[t];
    b += pb[t];
  }
  red[0][tid] = a;
  red[1][tid] = b;
  __syncthreads();
  for (int h = 128; h > 0; h >>= 1) {
    if (tid < h) {
      red[0][tid] += red[0][tid + h];
      red[1][tid] += red[1][tid + h];
    }
    __syncthreads();
  }
  if (tid != 0) return;
  const double mean = red[0][0] / (double)M;
  double var = red[1][0] / (double)M - mean * mean;
  if (var < 0.0) var = 0.0;
  mean_out[c] = (float)mean;
  invstd_out[c] = (float)(1.0 / sqrt(var + (double)eps));
  if (training && rm) {
    const double unb = M > 1 ? var * (double)M / (double)(M - 1) : var;
    rm[c] = (float)((1.0 - momentum) * rm[c] + momentum * mean);
    rv[c] = (float)((1.0 - momentum) * rv[c] + momentum * unb);
  }
}

hipError_t launch_bn_finalize_parts(const double *part, int ntiles, int C, int64_t M, float eps,
                                    float momentum, int training, float *rm, float *rv,
                                    float *mean_out, float *invstd_out, hipStream_t s,
                                    double *ys_zero, int nw) {
  if (!training) return hipErrorInvalidValue;
  hipLaunchKernelGGL(k_bn_finalize_parts, dim3(C), dim3(256), 0, s, part, ntiles, C, M, eps,
                     momentum, training, rm, rv, mean_out, invstd_out, ys_zero, nw);
  return hipGetLastError();
}

hipError_t launch_bn_finalize(const double *sum, const double *sq, int C, int64_t M, float eps,
                              float momentum, int training, float *rm, float *rv,
                              float *mean_out, float *invstd_out, hipStream_t s, unsigned *zw,
                              int nzw) {
  hipLaunchKernelGGL(k_bn_finalize, dim3((C + 255) / 256), dim3(256), 0, s, sum, sq, C, M, eps,
                     momentum, training, rm, rv, mean_out, invstd_out, zw, nzw);
  return hipGetLastError();
}

// y = ReLU(BN(U)); optionally (ysum != null) also the per-channel sum and sum
// of squares of y (fp64): the next block's BN1 batch statistics. A block
// covers kBnRows clips of one channel (one block reduction and one set of
// fp64 atomics per kBnRows rows: per-row blocks spent their time there).
// (y null, ABI 8: only the statistics -- the next block forms y itself from U,
// STGCN_PLAN_X_FROM_U -- as k_bn_relu_stats, so traces tell the two apart)
constexpr int kBnRows = 4;
template <int VEC, bool WY>
__device__ __forceinline__ void bn_relu_fwd_body(const float *U, const float *mean,
                                                 const float *invstd, const float *g,
                                                 const float *b, float *y, int N, int C, int L,
                                                 double *ysum, double *ysq, Dropout drop,
                                                 double *yext, unsigned *ymax) {
  __shared__ double red[8];
  const int c = blockIdx.x, n0 = blockIdx.y * kBnRows, n1 = min(N, n0 + kBnRows);
  const float mu = mean[c], is = invstd[c], a = is * g[c], be = b[c];
  double s = 0.0, q = 0.0, cnt = 0.0, su = 0.0, xu = 0.0;
  float ym = 0.f;  // max y (y >= 0): the next block's fp16 operand bound
  // (two vectors' loads issued before either's math; the sums stay fp64 per
  // element: the chain sums su / xu feed nearly cancelling BN2 backward terms)
  auto vec = [&](int64_t base, int i, float (&v)[VEC]) __attribute__((always_inline)) {
#pragma unroll
    for (int j = 0; j < VEC; ++j) {
      const float uh = (v[j] - mu) * is;
      const float t = (v[j] - mu) * a + be;
      v[j] = t > 0.f ? t : 0.f;
      if (drop.thresh) v[j] = dropout_keep(drop, base + i + j) ? v[j] * drop.scale : 0.f;
      s += (double)v[j];
      q += (double)v[j] * (double)v[j];
      ym = fmaxf(ym, v[j]);
      if (yext && t > 0.f) {
        cnt += 1.0;
        su += (double)uh;
        xu += (double)v[j] * (double)uh;
      }
    }
    if constexpr (WY) vst<VEC>(y + base + i, v);
  };
  for (int n = n0; n < n1; ++n) {
    const int64_t base = ((int64_t)n * C + c) * L;
    int i = threadIdx.x * VEC;
    for (; i + 256 * VEC < L; i += 512 * VEC) {
      float v0[VEC], v1[VEC];
      vld<VEC>(U + base + i, v0);
      vld<VEC>(U + base + i + 256 * VEC, v1);
      vec(base, i, v0);
      vec(base, i + 256 * VEC, v1);
    }
    if (i < L) {
      float v0[VEC];
      vld<VEC>(U + base + i, v0);
      vec(base, i, v0);
    }
  }
  if (ysum) block_sum2_atomic<256>(s, q, ysum + c, ysq + c, red);
  if (yext) {
    block_sum2_atomic<256>(cnt, su, yext + c, yext + C + c, red);
    block_sum2_atomic<256>(xu, 0.0, yext + 2 * C + c, nullptr, red);
  }
  if (ymax) block_amax<256>(ym, ymax);
}

template <int VEC>
__global__ __launch_bounds__(256) void k_bn_relu_fwd(const float *U, const float *mean,
                                                     const float *invstd, const float *g,
                                                     const float *b, float *y, int N, int C,
                                                     int L, double *ysum, double *ysq,
                                                     Dropout drop, double *yext,
                                                     unsigned *ymax) {
  bn_relu_fwd_body<VEC, true>(U, mean, invstd, g, b, y, N, C, L, ysum, ysq, drop, yext, ymax);
}

template <int VEC>
__global__ __launch_bounds__(256) void k_bn_relu_stats(const float *U, const float *mean,
                                                       const float *invstd, const float *g,
                                                       const float *b, float *y, int N, int C,
                                                       int L, double *ysum, double *ysq,
                                                       Dropout drop, double *yext,
                                                       unsigned *ymax) {
  bn_relu_fwd_body<VEC, false>(U, mean, invstd, g, b, y, N, C, L, ysum, ysq, drop, yext, ymax);
}

hipError_t launch_bn_relu_fwd(const float *U, const float *mean, const float *invstd,
                              const float *g, const float *b, float *y, int N, int C, int L,
                              double *ysum, double *ysq, Dropout drop, hipStream_t s,
                              double *yext, unsigned *ymax) {
  if (!y) {
    if (!ysum) return hipErrorInvalidValue;  // (nothing to form)
    STGCN_VEC_LAUNCH(k_bn_relu_stats, slice_vec(L, {U}), dim3(C, (N + kBnRows - 1) / kBnRows), U,
                     mean, invstd, g, b, y, N, C, L, ysum, ysq, drop, yext, ymax);
    return hipGetLastError();
  }
  STGCN_VEC_LAUNCH(k_bn_relu_fwd, slice_vec(L, {U, y}), dim3(C, (N + kBnRows - 1) / kBnRows), U,
                   mean, invstd, g, b, y, N, C, L, ysum, ysq, drop, yext, ymax);
  return hipGetLastError();
}

template <int VEC>
__global__ __launch_bounds__(256) void k_bn_relu_bwd_reduce(const float *dy, const float *U,
                                                            const float *mean,
                                                            const float *invstd, const float *g,
                                                            const float *b, int C, int L,
                                                            double *sg, double *sgu,
                                                            Dropout drop, const float *dync) {
  __shared__ double red[8];
  const int c = blockIdx.x, n = blockIdx.y;
  const int64_t base = ((int64_t)n * C + c) * L;
  const float mu = mean[c], is = invstd[c], a = is * g[c], be = b[c];
  const float dv = dync ? dync[(int64_t)n * C + c] : 0.f;  // (ABI 10: dy constant per row)
  double s = 0.0, q = 0.0;
  for (int i = threadIdx.x * VEC; i < L; i += 256 * VEC) {
    float u[VEC], d[VEC];
    vld<VEC>(U + base + i, u);
    if (dync) {
#pragma unroll
      for (int j = 0; j < VEC; ++j) d[j] = dv;
    } else {
      vld<VEC>(dy + base + i, d);
    }
    if (drop.thresh) {  // gradient through the fused dropout
#pragma unroll
      for (int j = 0; j < VEC; ++j)
        d[j] = dropout_keep(drop, base + i + j) ? d[j] * drop.scale : 0.f;
    }
#pragma unroll
    for (int j = 0; j < VEC; ++j) {
      if ((u[j] - mu) * a + be > 0.f) {
        s += d[j];
        q += (double)d[j] * (double)((u[j] - mu) * is);
      }
    }
  }
  block_sum2_atomic<256>(s, q, sg + c, sgu + c, red);
}

hipError_t launch_bn_relu_bwd_reduce(const float *dy, const float *U, const float *mean,
                                     const float *invstd, const float *g, const float *b, int N,
                                     int C, int L, double *sg, double *sgu, Dropout drop,
                                     hipStream_t s, const float *dync) {
  STGCN_VEC_LAUNCH(k_bn_relu_bwd_reduce, slice_vec(L, {dy, U}), dim3(C, N), dy, U, mean, invstd,
                   g, b, C, L, sg, sgu, drop, dync);
  return hipGetLastError();
}

template <int VEC>
__global__ __launch_bounds__(256) void k_bn_relu_bwd_apply(
    const float *dy, const float *U, const float *mean, const float *invstd, const float *g,
    const float *b, const double *sg, const double *sgu, float *dU, double *sdu, int C, int L,
    double invM, Dropout drop, int du_bf16, const float *dy_coef, const float *dync) {
  __shared__ double red[8];
  const int c = blockIdx.x, n = blockIdx.y;
  const int64_t base = ((int64_t)n * C + c) * L;
  const float dv = dync ? dync[(int64_t)n * C + c] : 0.f;  // (ABI 10: dy constant per row)
  const float mu = mean[c], is = invstd[c], a = is * g[c], be = b[c];
  const float mg = (float)(sg[c] * invM), mgu = (float)(sgu[c] * invM);
  // deferred dx of the next block: dy = ca * (dxhat - cmd - (y - cmu) * cis * cmdn)
  float ca = 0.f, cmd = 0.f, cmu = 0.f, cis = 0.f, cmdn = 0.f;
  if (dy_coef) {
    ca = dy_coef[c];
    cmd = dy_coef[C + c];
    cmu = dy_coef[2 * C + c];
    cis = dy_coef[3 * C + c];
    cmdn = dy_coef[4 * C + c];
  }
  double s = 0.0;
  for (int i = threadIdx.x * VEC; i < L; i += 256 * VEC) {
    float u[VEC], d[VEC], o[VEC];
    vld<VEC>(U + base + i, u);
    if (dync) {
#pragma unroll
      for (int j = 0; j < VEC; ++j) d[j] = dv;
    } else {
      vld<VEC>(dy + base + i, d);
    }
    if (dy_coef) {
#pragma unroll
      for (int j = 0; j < VEC; ++j) {
        const float t = (u[j] - mu) * a + be;
        const float yv = t > 0.f ? t : 0.f;  // this block's output, as k_bn_relu_fwd wrote it
        d[j] = ca * (d[j] - cmd - (yv - cmu) * cis * cmdn);
      }
    }
    if (drop.thresh) {
#pragma unroll
      for (int j = 0; j < VEC; ++j)
        d[j] = dropout_keep(drop, base + i + j) ? d[j] * drop.scale : 0.f;
    }
#pragma unroll
    for (int j = 0; j < VEC; ++j) {
      const float uh = (u[j] - mu) * is;
      const float gg = (u[j] - mu) * a + be > 0.f ? d[j] : 0.f;
      o[j] = a * (gg - mg - uh * mgu);
      s += o[j];
    }
    if (du_bf16) {  // dU stored in bf16 (its readers round it to bf16 anyway)
      __bf16 *ob = reinterpret_cast<__bf16 *>(dU) + base + i;
      unsigned short h[VEC];
#pragma unroll
      for (int j = 0; j < VEC; ++j) h[j] = __builtin_bit_cast(unsigned short, (__bf16)o[j]);
      if constexpr (VEC == 4)
        *reinterpret_cast<uint2 *>(ob) = make_uint2(h[0] | ((unsigned)h[1] << 16),
                                                    h[2] | ((unsigned)h[3] << 16));
      else if constexpr (VEC == 2)
        *reinterpret_cast<unsigned *>(ob) = h[0] | ((unsigned)h[1] << 16);
      else
        *reinterpret_cast<unsigned short *>(ob) = h[0];
    } else {
      vst<VEC>(dU + base + i, o);
    }
  }
  block_sum2_atomic<256>(s, 0.0, sdu + c, nullptr, red);
}

hipError_t launch_bn_relu_bwd_apply(const float *dy, const float *U, const float *mean,
                                    const float *invstd, const float *g, const float *b,
                                    const double *sg, const double *sgu, float *dU, double *sdu,
                                    int N, int C, int L, int training, Dropout drop,
                                    hipStream_t s, int du_bf16, const float *dy_coef,
                                    const float *dync) {
  // eval mode (constant running statistics): no batch-mean terms
  const double invM = training ? 1.0 / ((double)N * L) : 0.0;
  STGCN_VEC_LAUNCH(k_bn_relu_bwd_apply, slice_vec(L, {dy, U, dU}), dim3(C, N), dy, U, mean,
                   invstd, g, b, sg, sgu, dU, sdu, C, L, invM, drop, du_bf16, dy_coef, dync);
  return hipGetLastError();
}

// k_bn_relu_bwd_apply with the clip sums of its output (non-residual blocks):
// block = (channel c, 256 * VEC consecutive positions of the (T_out, V) row,
// clip chunk z), thread = VEC positions over the chunk's clips, so
// cs[z][c][pos] = sum_{n in chunk z} dU[n, c, pos] accumulates in registers
// (fp64, no atomics). Those sums give sum_{n,t} dZ by the per-tap algebra of
// kernels_fold.hip (SdZ = sum_q Wt_q^T Tq): the separate pass over dZ is gone.
template <int VEC>
__global__ __launch_bounds__(256) void k_bn_relu_bwd_apply_cols(
    const float *__restrict__ dy, const float *__restrict__ U, const float *mean,
    const float *invstd, const float *g, const float *b, const double *sg, const double *sgu,
    float *__restrict__ dU, double *sdu, int N, int C, int L, double invM, Dropout drop,
    int du_bf16, const float *dy_coef, double *__restrict__ cs, unsigned *amax,
    const float *dync) {
  __shared__ double red[8];
  float om = 0.f;  // max |dU| (f16x2 operand bound)
  const int c = blockIdx.x;
  const int i = (blockIdx.y * 256 + threadIdx.x) * VEC;
  const int nz = gridDim.z, per = (N + nz - 1) / nz;
  const int n0 = blockIdx.z * per, n1 = min(N, n0 + per);
  const float mu = mean[c], is = invstd[c], a = is * g[c], be = b[c];
  const float mg = (float)(sg[c] * invM), mgu = (float)(sgu[c] * invM);
  float ca = 0.f, cmd = 0.f, cmu = 0.f, cis = 0.f, cmdn = 0.f;
  if (dy_coef) {
    ca = dy_coef[c];
    cmd = dy_coef[C + c];
    cmu = dy_coef[2 * C + c];
    cis = dy_coef[3 * C + c];
    cmdn = dy_coef[4 * C + c];
  }
  double s = 0.0, col[VEC] = {};
  if (i < L) {
    // (two clips' operands in flight ahead of this clip's math and stores:
    // register sets A (even steps) and B (odd steps), loaded two clips ahead)
    float ua[VEC], da[VEC], ub[VEC], db[VEC];
    const int64_t cl = (int64_t)C * L;  // floats per clip
    const int64_t b0 = ((int64_t)n0 * C + c) * L + i;
    // (ABI 10, dync: dy constant over the row -- one value per clip, no dy tensor)
    auto ldy = [&](int64_t off, int nn, float (&dr)[VEC]) __attribute__((always_inline)) {
      if (dync) {
        const float dv = dync[(int64_t)nn * C + c];
#pragma unroll
        for (int j = 0; j < VEC; ++j) dr[j] = dv;
      } else {
        vld<VEC>(dy + off, dr);
      }
    };
    if (n0 < n1) {
      vld<VEC>(U + b0, ua);
      ldy(b0, n0, da);
    }
    if (n0 + 1 < n1) {
      vld<VEC>(U + b0 + cl, ub);
      ldy(b0 + cl, n0 + 1, db);
    }
    auto clip = [&](int n, float (&ur)[VEC], float (&dr)[VEC]) __attribute__((always_inline)) {
      const int64_t base = ((int64_t)n * C + c) * L;
      float u[VEC], d[VEC], o[VEC];
#pragma unroll
      for (int j = 0; j < VEC; ++j) {
        u[j] = ur[j];
        d[j] = dr[j];
      }
      if (n + 2 < n1) {
        vld<VEC>(U + base + 2 * cl + i, ur);
        ldy(base + 2 * cl + i, n + 2, dr);
      }
      if (dy_coef) {
#pragma unroll
        for (int j = 0; j < VEC; ++j) {
          const float t = (u[j] - mu) * a + be;
          const float yv = t > 0.f ? t : 0.f;
          d[j] = ca * (d[j] - cmd - (yv - cmu) * cis * cmdn);
        }
      }
      if (drop.thresh) {
#pragma unroll
        for (int j = 0; j < VEC; ++j)
          d[j] = dropout_keep(drop, base + i + j) ? d[j] * drop.scale : 0.f;
      }
#pragma unroll
      for (int j = 0; j < VEC; ++j) {
        const float uh = (u[j] - mu) * is;
        const float gg = (u[j] - mu) * a + be > 0.f ? d[j] : 0.f;
        o[j] = a * (gg - mg - uh * mgu);
        s += o[j];
        col[j] += o[j];
        om = fmaxf(om, fabsf(o[j]));
      }
      if (du_bf16) {
        __bf16 *ob = reinterpret_cast<__bf16 *>(dU) + base + i;
        unsigned short h[VEC];
#pragma unroll
        for (int j = 0; j < VEC; ++j) h[j] = __builtin_bit_cast(unsigned short, (__bf16)o[j]);
        if constexpr (VEC == 4)
          *reinterpret_cast<uint2 *>(ob) = make_uint2(h[0] | ((unsigned)h[1] << 16),
                                                      h[2] | ((unsigned)h[3] << 16));
        else if constexpr (VEC == 2)
          *reinterpret_cast<unsigned *>(ob) = h[0] | ((unsigned)h[1] << 16);
        else
          *reinterpret_cast<unsigned short *>(ob) = h[0];
      } else {
        vst<VEC>(dU + base + i, o);
      }
    };
    for (int n = n0; n < n1; n += 2) {
      clip(n, ua, da);
      if (n + 1 < n1) clip(n + 1, ub, db);
    }
#pragma unroll
    for (int j = 0; j < VEC; ++j) cs[((int64_t)blockIdx.z * C + c) * L + i + j] = col[j];
  }
  if (amax) block_amax<256>(om, amax);
  block_sum2_atomic<256>(s, 0.0, sdu + c, nullptr, red);
}

int apply_cols_chunks(int N) { return std::min(N, 4); }

// k_bn_relu_bwd_apply_cols for the folded block without G (capi.hip fold_bna).
// Block = (channel c, a tile of FR = 28 frames, clip chunk z), 256 threads; per
// clip of the chunk:
//   1. thread i < 252 takes joints 2i, 2i + 1 of the tile's 504 positions (fp32
//      pairs, coalesced): dU as k_bn_relu_bwd_apply_cols forms it, stored, its
//      clip-chunk sums in registers, and dU into an LDS row (double-buffered);
//   2. thread i forms dUA at positions e = i, i + 256 (< 504), frame e / V,
//      joint w = e % V:  dUA[n,c,t,w] = sum_v dU[n,c,t,v] A[v][w]  (fp32 fma in v
//      order, its two columns of A in registers), stored as coalesced words:
// the weight gradient's P operand. Also the fp16 operand bounds max |dU|
// (amax) and max |dUA| (amaxa). One barrier per clip.
constexpr int kFrTile = 28;
template <int V>
__global__ __launch_bounds__(256) void k_bn_relu_bwd_apply_fr(
    const float *__restrict__ dy, const float *__restrict__ U, const float *mean,
    const float *invstd, const float *g, const float *b, const double *sg, const double *sgu,
    float *__restrict__ dU, float *__restrict__ dUA, double *sdu, int N, int C, int To,
    double invM, Dropout drop, const float *dy_coef, double *__restrict__ cs, unsigned *amax,
    unsigned *amaxa, const float *A) {
  static_assert(V % 2 == 0, "whole pairs per frame");
  constexpr int NP = kFrTile * V;  // positions of a tile
  static_assert(NP / 2 <= 256 && NP <= 512, "one pair per thread, two outputs per thread");
  __shared__ float ob[2][NP];
  __shared__ double red[8];
  const int tid = threadIdx.x;
  const int c = blockIdx.x;
  const int f0 = blockIdx.y * kFrTile, nf = min(kFrTile, To - f0);
  const int L = To * V, np = nf * V;
  const int nz = gridDim.z, per = (N + nz - 1) / nz;
  const int n0 = blockIdx.z * per, n1 = min(N, n0 + per);
  const float mu = mean[c], is = invstd[c], a = is * g[c], be = b[c];
  const float mg = (float)(sg[c] * invM), mgu = (float)(sgu[c] * invM);
  float ca = 0.f, cmd = 0.f, cmu = 0.f, cis = 0.f, cmdn = 0.f;
  if (dy_coef) {
    ca = dy_coef[c];
    cmd = dy_coef[C + c];
    cmu = dy_coef[2 * C + c];
    cis = dy_coef[3 * C + c];
    cmdn = dy_coef[4 * C + c];
  }
  // this thread's two output positions of dUA and their columns of A
  const int e0 = tid, e1 = tid + 256;
  const int w0 = e0 % V, w1 = e1 % V, fr0 = e0 / V, fr1 = e1 / V;
  float a0[V], a1[V];
#pragma unroll
  for (int v = 0; v < V; ++v) {
    a0[v] = A[v * V + w0];
    a1[v] = A[v * V + w1];
  }
  const int pp = 2 * tid;  // this thread's pair of phase 1
  const bool pok = pp < np;
  float om = 0.f, oma = 0.f;
  double s = 0.0, col0 = 0.0, col1 = 0.0;
  for (int n = n0; n < n1; ++n) {
    const int64_t base = ((int64_t)n * C + c) * L + (int64_t)f0 * V;
    float *obn = ob[(n - n0) & 1];
    if (pok) {
      const float2 uu = *reinterpret_cast<const float2 *>(U + base + pp);
      const float2 dd = *reinterpret_cast<const float2 *>(dy + base + pp);
      float u[2] = {uu.x, uu.y}, d[2] = {dd.x, dd.y}, o[2];
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        if (dy_coef) {
          const float tt = (u[j] - mu) * a + be;
          const float yv = tt > 0.f ? tt : 0.f;
          d[j] = ca * (d[j] - cmd - (yv - cmu) * cis * cmdn);
        }
        if (drop.thresh) d[j] = dropout_keep(drop, base + pp + j) ? d[j] * drop.scale : 0.f;
        const float uh = (u[j] - mu) * is;
        const float gg = (u[j] - mu) * a + be > 0.f ? d[j] : 0.f;
        o[j] = a * (gg - mg - uh * mgu);
        s += o[j];
        om = fmaxf(om, fabsf(o[j]));
      }
      col0 += o[0];
      col1 += o[1];
      *reinterpret_cast<float2 *>(dU + base + pp) = make_float2(o[0], o[1]);
      *reinterpret_cast<float2 *>(obn + pp) = make_float2(o[0], o[1]);
    }
    __syncthreads();  // (double buffer: the other row is free since the last barrier)
    if (e0 < np) {
      const float *r = obn + fr0 * V;
      float t = r[0] * a0[0];
#pragma unroll
      for (int v = 1; v < V; ++v) t = fmaf(r[v], a0[v], t);
      dUA[base + e0] = t;
      oma = fmaxf(oma, fabsf(t));
    }
    if (e1 < np) {
      const float *r = obn + fr1 * V;
      float t = r[0] * a1[0];
#pragma unroll
      for (int v = 1; v < V; ++v) t = fmaf(r[v], a1[v], t);
      dUA[base + e1] = t;
      oma = fmaxf(oma, fabsf(t));
    }
  }
  if (pok) {
    double *dst = cs + ((int64_t)blockIdx.z * C + c) * L + (int64_t)f0 * V + pp;
    dst[0] = col0;
    dst[1] = col1;
  }
  block_amax<256>(om, amax);
  __syncthreads();  // (block_amax's LDS words are reused by the second call)
  block_amax<256>(oma, amaxa);
  block_sum2_atomic<256>(s, 0.0, sdu + c, nullptr, red);
}

hipError_t launch_bn_relu_bwd_apply_fr(const float *dy, const float *U, const float *mean,
                                       const float *invstd, const float *g, const float *b,
                                       const double *sg, const double *sgu, float *dU, float *dUA,
                                       double *sdu, int N, int C, int To, int V, int training,
                                       Dropout drop, const float *dy_coef, double *cs,
                                       unsigned *amax, unsigned *amaxa, const float *A,
                                       hipStream_t s) {
  if (V != 18 || !amax || !amaxa || !A) return hipErrorInvalidValue;
  const double invM = training ? 1.0 / ((double)N * To * V) : 0.0;
  hipLaunchKernelGGL((k_bn_relu_bwd_apply_fr<18>),
                     dim3(C, (To + kFrTile - 1) / kFrTile, apply_cols_chunks(N)), dim3(256), 0, s,
                     dy, U, mean, invstd, g, b, sg, sgu, dU, dUA, sdu, N, C, To, invM, drop, dy_coef,
                     cs, amax, amaxa, A);
  return hipGetLastError();
}

hipError_t launch_bn_relu_bwd_apply_cols(const float *dy, const float *U, const float *mean,
                                         const float *invstd, const float *g, const float *b,
                                         const double *sg, const double *sgu, float *dU,
                                         double *sdu, int N, int C, int L, int training,
                                         Dropout drop, hipStream_t s, int du_bf16,
                                         const float *dy_coef, double *cs, unsigned *amax,
                                         const float *dync) {
  const double invM = training ? 1.0 / ((double)N * L) : 0.0;
  // (whole-row vectors: every row start VEC-aligned needs L % VEC == 0)
  int vec = slice_vec(L, {dy, U, dU});
  const int nz = apply_cols_chunks(N);
#define COLS_LAUNCH(VV)                                                                     \
  hipLaunchKernelGGL((k_bn_relu_bwd_apply_cols<VV>), dim3(C, (L + 256 * VV - 1) / (256 * VV), nz), \
                     dim3(256), 0, s, dy, U, mean, invstd, g, b, sg, sgu, dU, sdu, N, C, L,  \
                     invM, drop, du_bf16, dy_coef, cs, amax, dync)
  if (vec == 4)
    COLS_LAUNCH(4);
  else if (vec == 2)
    COLS_LAUNCH(2);
  else
    COLS_LAUNCH(1);
#undef COLS_LAUNCH
  return hipGetLastError();
}

// The deferred-dx chain's per-channel finalize (see internal.h): with
// a = invstd1 g1, md = sd / M, mdn = sdn / M the next-to-be-applied dx is
//   dx = a (dxhat - md - (x - mu1) invstd1 mdn)
// and, x = ReLU(g2 uhat + b2) being the previous block's output (x = 0 off its
// mask m), the previous block's ReLU+BN2 backward sums follow from the prev-mode
// sums s1 = sum m dxhat, s2 = sum m dxhat uhat and that block's forward sums
// (cnt = sum m, su = sum m uhat, sum x, xu = sum x uhat):
//   sum m dx       = a (s1 - md cnt - mdn invstd1 (sum x - mu1 cnt))
//   sum m dx uhat  = a (s2 - md su  - mdn invstd1 (xu    - mu1 su))
__global__ void k_chain_coef(const double *sd, const double *sdn, const float *mean1,
                             const float *invstd1, const float *g1, const double *s1,
                             const double *s2, const double *xst, int C, double invM,
                             float *dg1, float *db1, float *coef, double *psum) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  const double md = sd[c] * invM, mdn = sdn[c] * invM;
  const float af = invstd1[c] * g1[c];
  const double a = (double)af, is = (double)invstd1[c], mu = (double)mean1[c];
  const double sx = xst[c], cnt = xst[2 * C + c], su = xst[3 * C + c], xu = xst[4 * C + c];
  dg1[c] = (float)sdn[c];
  db1[c] = (float)sd[c];
  coef[c] = af;
  coef[C + c] = (float)md;
  coef[2 * C + c] = mean1[c];
  coef[3 * C + c] = invstd1[c];
  coef[4 * C + c] = (float)mdn;
  psum[c] = a * (s1[c] - md * cnt - mdn * is * (sx - mu * cnt));
  psum[C + c] = a * (s2[c] - md * su - mdn * is * (xu - mu * su));
}

hipError_t launch_chain_coef(const double *sd, const double *sdn, const float *mean1,
                             const float *invstd1, const float *g1, const double *s1,
                             const double *s2, const double *xst, int C, int64_t M,
                             float *dg1, float *db1, float *coef, double *psum, hipStream_t s) {
  hipLaunchKernelGGL(k_chain_coef, dim3((C + 255) / 256), dim3(256), 0, s, sd, sdn, mean1,
                     invstd1, g1, s1, s2, xst, C, 1.0 / (double)M, dg1, db1, coef, psum);
  return hipGetLastError();
}

__global__ void k_bn_grads_out(const double *sg, const double *sgu, const double *sdu, int C,
                               float *dgamma, float *dbeta, float *dbias) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  dgamma[c] = (float)sgu[c];
  dbeta[c] = (float)sg[c];
  if (dbias) dbias[c] = (float)sdu[c];
}

hipError_t launch_bn_grads_out(const double *sg, const double *sgu, const double *sdu, int C,
                               float *dgamma, float *dbeta, float *dbias, hipStream_t s) {
  hipLaunchKernelGGL(k_bn_grads_out, dim3((C + 255) / 256), dim3(256), 0, s, sg, sgu, sdu, C,
                     dgamma, dbeta, dbias);
  return hipGetLastError();
}

// dx = g*invstd * (dxhat - sum(dxhat)/M - xnorm * sum(dxhat*xnorm)/M), in place
// (invM = 0: eval mode, constant running statistics -> dx = g*invstd*dxhat).
// Optionally (pg2 != null) also the previous block's ReLU+BN2 backward sums:
// x = ReLU(g2*uhat + b2) of that block, so its ReLU mask is x > 0 and
// uhat = (x - b2) / g2 there; with dy_prev = dx:
//   psum[c] += sum dx * [x > 0],  psum[C + c] += sum dx * [x > 0] * uhat.
// The division loses precision when |b2| >> |g2| (and is undefined at g2 = 0):
// for such channels (|b2| > 4|g2|, a channel-uniform branch) uhat is read from
// the previous block's saved pre-BN2 tensor pU instead, exactly as that
// block's own reduction computes it: uhat = (U - mean2) * invstd2, mask
// (U - mean2) * invstd2*g2 + b2 > 0.
template <int VEC>
__global__ __launch_bounds__(256) void k_bn1_bwd_apply(float *dx, const float *x,
                                                       const float *mean, const float *invstd,
                                                       const float *g, const double *sd,
                                                       const double *sdn, const float *add,
                                                       int C, int L, double invM,
                                                       const float *pg2, const float *pb2,
                                                       double *psum, const float *pU,
                                                       const float *pmean, const float *pinvstd) {
  __shared__ double red[8];
  const int c = blockIdx.x, n = blockIdx.y;
  const int64_t base = ((int64_t)n * C + c) * L;
  const float mu = mean[c], is = invstd[c], a = is * g[c];
  const float md = (float)(sd[c] * invM), mdn = (float)(sdn[c] * invM);
  const float pg = pg2 ? pg2[c] : 1.f, pb = pg2 ? pb2[c] : 0.f;
  // poorly conditioned reconstruction (or g2 == 0 / non-finite): use U
  const bool from_u = pg2 && pU && !(fabsf(pb) <= 4.f * fabsf(pg));
  const float pmu = from_u ? pmean[c] : 0.f, pis = from_u ? pinvstd[c] : 1.f;
  const float pa = pis * pg;
  double s = 0.0, q = 0.0;
  for (int i = threadIdx.x * VEC; i < L; i += 256 * VEC) {
    float xv[VEC], d[VEC];
    vld<VEC>(x + base + i, xv);
    vld<VEC>(dx + base + i, d);
#pragma unroll
    for (int j = 0; j < VEC; ++j) d[j] = a * (d[j] - md - (xv[j] - mu) * is * mdn);
    if (add) {
      float r[VEC];
      vld<VEC>(add + base + i, r);
#pragma unroll
      for (int j = 0; j < VEC; ++j) d[j] += r[j];
    }
    vst<VEC>(dx + base + i, d);
    if (from_u) {
      float u[VEC];
      vld<VEC>(pU + base + i, u);
#pragma unroll
      for (int j = 0; j < VEC; ++j)
        if ((u[j] - pmu) * pa + pb > 0.f) {
          s += d[j];
          q += (double)d[j] * (double)((u[j] - pmu) * pis);
        }
    } else if (pg2) {
#pragma unroll
      for (int j = 0; j < VEC; ++j)
        if (xv[j] > 0.f) {
          s += d[j];
          q += (double)d[j] * (double)((xv[j] - pb) / pg);
        }
    }
  }
  if (pg2) block_sum2_atomic<256>(s, q, psum + c, psum + C + c, red);
}

hipError_t launch_bn1_bwd_apply(float *dx, const float *x, const float *mean, const float *invstd,
                                const float *g, const double *sd, const double *sdn,
                                const float *add, int N, int C, int L, int64_t M, int training,
                                const float *pg2, const float *pb2, double *psum,
                                const float *pU, const float *pmean, const float *pinvstd,
                                hipStream_t s) {
  STGCN_VEC_LAUNCH(k_bn1_bwd_apply, slice_vec(L, {dx, x, add, pU}), dim3(C, N), dx, x, mean,
                   invstd, g, sd, sdn, add, C, L, training ? 1.0 / (double)M : 0.0, pg2, pb2,
                   psum, pU, pmean, pinvstd);
  return hipGetLastError();
}

// dout = dy * (y > 0) for the residual block's final ReLU (st_graphconv.py:105),
// with the per-channel sum of dout (the temporal and projection bias grads).
template <int VEC>
__global__ __launch_bounds__(256) void k_relu_bwd(const float *dy, const float *y, float *dout,
                                                  double *sum, int C, int L, float scale) {
  __shared__ double red[8];
  const int c = blockIdx.x, n = blockIdx.y;
  const int64_t base = ((int64_t)n * C + c) * L;
  double s = 0.0;
  for (int i = threadIdx.x * VEC; i < L; i += 256 * VEC) {
    float d[VEC], yv[VEC];
    vld<VEC>(dy + base + i, d);
    vld<VEC>(y + base + i, yv);
#pragma unroll
    for (int j = 0; j < VEC; ++j) {
      d[j] = yv[j] > 0.f ? d[j] * scale : 0.f;
      s += d[j];
    }
    vst<VEC>(dout + base + i, d);
  }
  block_sum2_atomic<256>(s, 0.0, sum + c, nullptr, red);
}

hipError_t launch_relu_bwd(const float *dy, const float *y, float *dout, double *sum, int N,
                           int C, int L, float scale, hipStream_t s) {
  STGCN_VEC_LAUNCH(k_relu_bwd, slice_vec(L, {dy, y, dout}), dim3(C, N), dy, y, dout, sum, C, L,
                   scale);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// Spatial (graph) kernels.
// ---------------------------------------------------------------------------
__global__ void k_pack_w(const float *W, float *Wpk, int K, int R, int C) {
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;  // co*(K*C) + k*C + ci
  const int KC = K * C;
  if (idx >= R * KC) return;
  const int co = idx / KC, rem = idx - co * KC, k = rem / C, ci = rem - k * C;
  Wpk[idx] = W[((int64_t)k * R + co) * C + ci];
}

hipError_t launch_pack_w(const float *W, float *Wpk, int K, int R, int C, hipStream_t s) {
  const int n = R * K * C;
  hipLaunchKernelGGL(k_pack_w, dim3((n + 255) / 256), dim3(256), 0, s, W, Wpk, K, R, C);
  return hipGetLastError();
}

// bias_rv[co][v] = sum_k bW[k*R+co] * sum_w A[k][v][w]   (the 1x1-conv bias
// pushed through the joint contraction: st_graphconv.py:148-150)
__global__ void k_bias_rv(const float *A, const float *bW, float *bias_rv, int K, int R, int V) {
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= R * V) return;
  const int co = idx / V, v = idx - co * V;
  double s = 0.0;
  for (int k = 0; k < K; ++k) {
    double ra = 0.0;
    for (int w = 0; w < V; ++w) ra += A[((int64_t)k * V + v) * V + w];
    s += (double)bW[k * R + co] * ra;
  }
  bias_rv[idx] = (float)s;
}

hipError_t launch_bias_rv(const float *A, const float *bW, float *bias_rv, int K, int R, int V,
                          hipStream_t s) {
  hipLaunchKernelGGL(k_bias_rv, dim3((R * V + 255) / 256), dim3(256), 0, s, A, bW, bias_rv, K, R,
                     V);
  return hipGetLastError();
}

constexpr int kGatherTC = 32;  // frames per gather block

// G[n][k*C+ci][t][v] = sum_w A[k][v][w] * BN1(x)[n][ci][t][w]
// One block per (n, frame chunk); A pinned in LDS; loop over channels.
__global__ __launch_bounds__(256) void k_gather_fwd(const float *x, const float *mean,
                                                    const float *invstd, const float *g,
                                                    const float *b, const float *A, float *G,
                                                    int C, int T, int V, int K, int relu,
                                                    unsigned *amax) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float *As = smem;                 // [K][V][V]
  float gm = 0.f;
  float *xs = smem + K * V * V;     // [TC][V]
  const int n = blockIdx.y, t0 = blockIdx.x * kGatherTC;
  int tc = T - t0;
  if (tc > kGatherTC) tc = kGatherTC;
  for (int i = threadIdx.x; i < K * V * V; i += 256) As[i] = A[i];
  const int L = T * V;
  const int nout = K * tc * V;
  for (int ci = 0; ci < C; ++ci) {
    __syncthreads();
    const float *src = x + ((int64_t)n * C + ci) * L + (int64_t)t0 * V;
    const float mu = mean[ci], a = invstd[ci] * g[ci], be = b[ci];
    for (int i = threadIdx.x; i < tc * V; i += 256) {
      const float t = (src[i] - mu) * a + be;
      xs[i] = relu ? fmaxf(t, 0.f) : t;
    }
    __syncthreads();
    for (int o = threadIdx.x; o < nout; o += 256) {
      const int k = o / (tc * V);
      const int rem = o - k * tc * V;
      const int t = rem / V, v = rem - t * V;
      const float *ar = As + (k * V + v) * V;
      const float *xr = xs + t * V;
      float s = 0.f;
      for (int w = 0; w < V; ++w) s = fmaf(ar[w], xr[w], s);
      G[(((int64_t)n * K + k) * C + ci) * L + (int64_t)(t0 + t) * V + v] = s;
      gm = fmaxf(gm, fabsf(s));
    }
  }
  if (amax) block_amax<256>(gm, amax);
}

// Joint-axis (V) kernels: rows padded to VP (multiple of 4) for 16-byte LDS reads.
template <int V>
struct JointCfg {
  static constexpr int VP = (V + 3) & ~3;
};

// ---------------------------------------------------------------------------
// Flat row-parallel joint kernels: one thread per (n, ci, t) row of the whole
// tensor (rows are contiguous in NCTV memory), RB rows per workgroup, no
// per-slice chunk loop. A sits in LDS ([K][V][VP], 16-B broadcast reads).
// ---------------------------------------------------------------------------
template <int V>
__global__ __launch_bounds__(256) void k_gather3(const float *__restrict__ x,
                                                 const float *__restrict__ mean,
                                                 const float *__restrict__ invstd,
                                                 const float *__restrict__ g,
                                                 const float *__restrict__ b,
                                                 const float *__restrict__ A, float *G, int C,
                                                 int T, int K, int64_t rows, int relu,
                                                 unsigned *amax) {
  constexpr int VP = JointCfg<V>::VP;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float *As = smem;  // [K][V][VP]
  const int tid = threadIdx.x;
  for (int i = tid; i < K * V * VP; i += blockDim.x) {
    const int kv = i / VP, w = i - kv * VP;
    As[i] = w < V ? A[kv * V + w] : 0.f;
  }
  __syncthreads();
  const int64_t r0 = (int64_t)blockIdx.x * blockDim.x + tid;
  const bool live = r0 < rows;
  const int64_t r = live ? r0 : rows - 1;  // (the last row again: every lane reaches wave_amax)
  float gm = 0.f;
  const int64_t CT = (int64_t)C * T;
  const int64_t n = r / CT;
  const int rem = (int)(r - n * CT);
  const int ci = rem / T, t = rem - ci * T;
  const float mu = mean[ci], a = invstd[ci] * g[ci], be = b[ci];
  const float *xr = x + r * V;
  float xv[VP];
#pragma unroll
  for (int w = 0; w < VP; ++w) {
    const float t = w < V ? (xr[w] - mu) * a + be : 0.f;
    xv[w] = relu ? fmaxf(t, 0.f) : t;
  }
  for (int k = 0; k < K; ++k) {
    float *gout = G + ((n * K + k) * C + ci) * (int64_t)T * V + (int64_t)t * V;
    const float *Ak = As + k * V * VP;
#pragma unroll
    for (int v = 0; v < V; ++v) {
      float acc = 0.f;
#pragma unroll
      for (int w4 = 0; w4 < VP; w4 += 4) {
        const float4 q = *reinterpret_cast<const float4 *>(Ak + v * VP + w4);
        acc = fmaf(q.x, xv[w4], acc);
        acc = fmaf(q.y, xv[w4 + 1], acc);
        acc = fmaf(q.z, xv[w4 + 2], acc);
        acc = fmaf(q.w, xv[w4 + 3], acc);
      }
      if (live) gout[v] = acc;
      gm = fmaxf(gm, fabsf(acc));
    }
  }
  if (amax) block_amax<256>(gm, amax);
}

// k_gather4: k_gather3 with the block's rows moved through LDS: the 256 rows
// of a block are contiguous in x (256*V floats; the host checks that no block
// crosses a clip, so each partition's 256*V outputs are contiguous in G too),
// they arrive by 16-byte LDS-DMA, each thread contracts its row from LDS (A in
// LDS), and the outputs leave through LDS as float4 stores. (A persistent,
// double-buffered variant measured slower: fewer workgroups per CU.)
// pv.mean non-null (ABI 8, STGCN_PLAN_X_FROM_U): x holds the previous block's U
// and the input is ReLU(BN2_prev(U)), formed as k_bn_relu_fwd forms its y.
template <int V>
__global__ __launch_bounds__(256) void k_gather4(const float *__restrict__ x,
                                                 const float *__restrict__ mean,
                                                 const float *__restrict__ invstd,
                                                 const float *__restrict__ g,
                                                 const float *__restrict__ b,
                                                 const float *__restrict__ A, float *G, int C,
                                                 int T, int K, int64_t rows, int relu,
                                                 unsigned *amax, PrevBn pv) {
  constexpr int VP = JointCfg<V>::VP;
  constexpr int BF = 256 * V;  // floats of a block (a multiple of 256: V DMA rounds)
  float gm = 0.f;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  float *xs = smem;     // [256][V]
  float *os = xs + BF;  // [256][V]
  float *As = os + BF;  // [K][V][VP]
  const int64_t r0 = (int64_t)blockIdx.x * 256;
  {
    const __amdgpu_buffer_rsrc_t rs = make_rsrc(x + r0 * V, BF);
    for (int i = wave; i < V; i += 4)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, xs + i * 256, 16, (unsigned)(i * 256 + lane * 4) * 4u,
                                               0, 0, 0);
  }
  for (int i = tid; i < K * V * VP; i += 256) {
    const int kv = i / VP, w = i - kv * VP;
    As[i] = w < V ? A[kv * V + w] : 0.f;
  }
  const int64_t CT = (int64_t)C * T;
  const int64_t n0 = r0 / CT, rem0 = r0 - n0 * CT;
  const int ci = (int)((rem0 + tid) / T);
  const float mu = mean[ci], a = invstd[ci] * g[ci], be = b[ci];
  const bool prev = pv.mean != nullptr;
  const float pmu = prev ? pv.mean[ci] : 0.f, pa = prev ? pv.invstd[ci] * pv.g[ci] : 0.f;
  const float pbe = prev ? pv.b[ci] : 0.f;
  __syncthreads();
  float xv[VP];
#pragma unroll
  for (int w = 0; w < VP; ++w) {
    float xx = w < V ? xs[tid * V + w] : 0.f;
    if (prev) {
      const float u = (xx - pmu) * pa + pbe;
      xx = u > 0.f ? u : 0.f;
    }
    const float t = w < V ? (xx - mu) * a + be : 0.f;
    xv[w] = relu ? fmaxf(t, 0.f) : t;
  }
  for (int k = 0; k < K; ++k) {
    const float *Ak = As + k * V * VP;
    if (k > 0) __syncthreads();  // previous partition's stores have read os
#pragma unroll
    for (int v = 0; v < V; ++v) {
      float acc = 0.f;
#pragma unroll
      for (int w4 = 0; w4 < VP; w4 += 4) {
        const float4 q = *reinterpret_cast<const float4 *>(Ak + v * VP + w4);
        acc = fmaf(q.x, xv[w4], acc);
        acc = fmaf(q.y, xv[w4 + 1], acc);
        acc = fmaf(q.z, xv[w4 + 2], acc);
        acc = fmaf(q.w, xv[w4 + 3], acc);
      }
      os[tid * V + v] = acc;
    }
    __syncthreads();
    float *dst = G + ((n0 * K + k) * CT + rem0) * V;
    for (int e = tid; e < BF / 4; e += 256) {
      const float4 q = *reinterpret_cast<const float4 *>(os + e * 4);
      *reinterpret_cast<float4 *>(dst + e * 4) = q;
      gm = fmaxf(gm, fmaxf(fmaxf(fabsf(q.x), fabsf(q.y)), fmaxf(fabsf(q.z), fabsf(q.w))));
    }
  }
  if (amax) block_amax<256>(gm, amax);
}

// Flat-row spatial backward (the math: see k_spatial_dx). Per block:
// dx rows, BN1 sums reduced per channel segment in LDS (rows are sorted by
// channel), dA over the block's rows on MFMA, wave partials summed in LDS.
template <int V>
__global__ __launch_bounds__(256) void k_spatial_bwd3(
    const float *__restrict__ H, const float *__restrict__ x, const float *__restrict__ mean,
    const float *__restrict__ invstd, const float *__restrict__ g, const float *__restrict__ b,
    const float *__restrict__ A, float *dx, float *dA, double *sd, double *sdn, int C, int T,
    int K, int64_t rows, int write_dx, int relu, float *dA_part) {
  constexpr int VP = JointCfg<V>::VP;
  constexpr int NT = (V + 31) / 32;
  constexpr int MAXSEG = 32;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  __shared__ double seg_s[MAXSEG], seg_n[MAXSEG];
  const int RB = blockDim.x;
  float *As = smem;                 // [K][V][VP]
  float *Hs = As + K * V * VP;      // [K][RB][V]
  float *XBs = Hs + K * RB * V;     // [RB][VP] BN1(x)
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, hi = lane >> 5, lo = lane & 31;
  for (int i = tid; i < K * V * VP; i += RB) {
    const int kv = i / VP, w = i - kv * VP;
    As[i] = w < V ? A[kv * V + w] : 0.f;
  }
  if (tid < MAXSEG) seg_s[tid] = seg_n[tid] = 0.0;
  const int64_t r0 = (int64_t)blockIdx.x * RB;
  const int64_t r = r0 + tid;
  const bool live = r < rows;
  const int64_t CT = (int64_t)C * T;
  // channel segment of this row relative to the block's first row
  const int64_t cfirst = (r0 / CT) * C + (int)((r0 % CT) / T);  // global (n*C + ci) of row r0
  int64_t n = 0;
  int ci = 0, t = 0;
  if (live) {
    n = r / CT;
    const int rem = (int)(r - n * CT);
    ci = rem / T;
    t = rem - ci * T;
  }
  const int seg = live ? (int)((n * C + ci) - cfirst) : 0;
  const bool seg_lds = (RB + T - 1) / T + 1 <= MAXSEG;
  __syncthreads();
  float s = 0.f, sn = 0.f;
  if (live) {
    const float mu = mean[ci], is = invstd[ci], a = is * g[ci], be = b[ci];
    const float *xr = x + r * V;
    float xv[VP];
#pragma unroll
    for (int w = 0; w < VP; ++w) xv[w] = w < V ? xr[w] : 0.f;
    float acc[VP];
#pragma unroll
    for (int w = 0; w < VP; ++w) acc[w] = 0.f;
    for (int k = 0; k < K; ++k) {
      const float *hr = H + ((n * K + k) * C + ci) * (int64_t)T * V + (int64_t)t * V;
      const float *Ak = As + k * V * VP;
#pragma unroll
      for (int v = 0; v < V; ++v) {
        const float h = hr[v];
        Hs[(k * RB + tid) * V + v] = h;
#pragma unroll
        for (int w4 = 0; w4 < VP; w4 += 4) {
          const float4 q = *reinterpret_cast<const float4 *>(Ak + v * VP + w4);
          acc[w4] = fmaf(h, q.x, acc[w4]);
          acc[w4 + 1] = fmaf(h, q.y, acc[w4 + 1]);
          acc[w4 + 2] = fmaf(h, q.z, acc[w4 + 2]);
          acc[w4 + 3] = fmaf(h, q.w, acc[w4 + 3]);
        }
      }
    }
    float *dxr = dx + r * V;
#pragma unroll
    for (int w = 0; w < V; ++w) {
      const float xn = (xv[w] - mu) * is;
      const float bn = (xv[w] - mu) * a + be;
      if (relu && bn <= 0.f) acc[w] = 0.f;  // ReLU'(BN1(x))
      s += acc[w];
      sn = fmaf(acc[w], xn, sn);
      if (write_dx) dxr[w] = acc[w];
      XBs[tid * VP + w] = relu ? fmaxf(bn, 0.f) : bn;
    }
  } else {
    for (int k = 0; k < K; ++k)
#pragma unroll
      for (int v = 0; v < V; ++v) Hs[(k * RB + tid) * V + v] = 0.f;
#pragma unroll
    for (int w = 0; w < V; ++w) XBs[tid * VP + w] = 0.f;
  }
  // BN1 partial sums per channel segment
  if (seg_lds) {
    if (live) {
      atomicAdd(&seg_s[seg], (double)s);
      atomicAdd(&seg_n[seg], (double)sn);
    }
  } else if (live) {
    atomicAdd(sd + ci, (double)s);
    atomicAdd(sdn + ci, (double)sn);
  }
  __syncthreads();
  if (seg_lds && tid < MAXSEG) {
    const int64_t gc = cfirst + tid;  // global (n*C + ci)
    const int64_t rlast = min(r0 + RB, rows) - 1;
    const int64_t glast = (rlast / CT) * C + (int)((rlast % CT) / T);
    if (gc <= glast) {
      const int cc = (int)(gc % C);
      atomicAdd(sd + cc, seg_s[tid]);
      atomicAdd(sdn + cc, seg_n[tid]);
    }
  }
  // dA on MFMA over the block's rows (wave takes row pairs kk = wave, +nw, ...);
  // each wave's tiles go to its own slice [wave][K][DW][DW] (one owner lane per
  // entry: plain stores), summed over the waves in wave order below
  const int nw = RB / 64;
  const int nk = RB / 2;
  const int DW = NT * 32;
  float *dred = XBs + RB * VP + wave * K * DW * DW;
  __syncthreads();
  for (int k = 0; k < K; ++k) {
    floatx16 dacc[NT][NT];
#pragma unroll
    for (int p2 = 0; p2 < NT; ++p2)
#pragma unroll
      for (int q2 = 0; q2 < NT; ++q2)
#pragma unroll
        for (int i = 0; i < 16; ++i) dacc[p2][q2][i] = 0.f;
    const float *hk = Hs + k * RB * V;
    for (int kk = wave; kk < nk; kk += nw) {
      const int rr = 2 * kk + hi;
#pragma unroll
      for (int p2 = 0; p2 < NT; ++p2) {
        const int v = p2 * 32 + lo;
        const float av = v < V ? hk[rr * V + v] : 0.f;
#pragma unroll
        for (int q2 = 0; q2 < NT; ++q2) {
          const int w = q2 * 32 + lo;
          const float bw = w < V ? XBs[rr * VP + w] : 0.f;
          dacc[p2][q2] = mfma32(av, bw, dacc[p2][q2]);
        }
      }
    }
#pragma unroll
    for (int p2 = 0; p2 < NT; ++p2)
#pragma unroll
      for (int q2 = 0; q2 < NT; ++q2)
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const int v = p2 * 32 + (i & 3) + 8 * (i >> 2) + 4 * hi;
          const int w = q2 * 32 + lo;
          if (v < V && w < V) dred[(k * DW + v) * DW + w] = dacc[p2][q2][i];
        }
  }
  __syncthreads();
  const float *dw0 = XBs + RB * VP;
  for (int i = tid; i < K * V * V; i += RB) {
    const int k = i / (V * V), rem = i - k * V * V, v = rem / V, w = rem - v * V;
    float sum = 0.f;
    for (int wv = 0; wv < nw; ++wv) sum += dw0[((wv * K + k) * DW + v) * DW + w];
    if (dA_part)  // (deterministic: launch_dA_reduce adds the partials in order)
      dA_part[(int64_t)blockIdx.x * K * V * V + i] = sum;
    else
      atomicAdd(dA + i, sum);
  }
}

// Row-pass sums of k_spatial_bwd5 / _bwd6 (float sv[4]: sd, sdn and, in prev
// mode, s1, s2 of PrevBn; ns of them), reduced per channel segment of the
// block: a wave whose rows share one channel reduces once; LDS segment
// accumulators (the kernel's __shared__ segv[4][MAXSEG]) when the block spans
// few channels, else global fp64 atomics. (A macro: the LDS array must stay a
// visible __shared__ object at the atomics, or hipcc mis-selects them.)
#define STGCN_ROWPASS_SUMS(sv, ns, seg, ci)                                   \
  do {                                                                        \
    const int seg0_ = __builtin_amdgcn_readfirstlane(seg);                    \
    if (__builtin_amdgcn_ballot_w64((seg) != seg0_) == 0) {                   \
      for (int i_ = 0; i_ < (ns); ++i_) {                                     \
        const double w_ = wave_sum((double)(sv)[i_]);                         \
        if (lane == 0) {                                                      \
          if (seg_lds)                                                        \
            atomicAdd(&segv[i_][seg0_], w_);                                  \
          else                                                                \
            atomicAdd(gdst[i_] + (ci), w_);                                   \
        }                                                                     \
      }                                                                       \
    } else {                                                                  \
      for (int i_ = 0; i_ < (ns); ++i_) {                                     \
        if (seg_lds)                                                          \
          atomicAdd(&segv[i_][seg], (double)(sv)[i_]);                        \
        else                                                                  \
          atomicAdd(gdst[i_] + (ci), (double)(sv)[i_]);                       \
      }                                                                       \
    }                                                                         \
  } while (0)

// k_spatial_bwd5: the spatial backward with both joint contractions on MFMA.
// Persistent and double-buffered like k_spatial_bwd4 (row blocks of RB rows,
// contiguous in x, dx and per partition in H; H planes and x by 16-byte
// LDS-DMA). Per block:
//   dx[row][w] = sum_k sum_v H_k[row][v] A_k[v][w]   MFMA, A_k resident in VGPRs
//                                                    as the B operand (k = v)
//   BN1 sums per row from the dx tile in LDS, BN1(x) in place (one thread/row)
//   dA_k[v][w] += sum_rows H_k[row][v] BN1(x)[row][w]  MFMA, LDS accumulator
// dx leaves through LDS as float4 stores. With 3 partitions, 8 waves (two per
// SIMD): wave w takes dx row tile w & 3 (if < RB/32) over half w >> 2 of the
// joint reduction (the halves meet in LDS and are summed by the row pass), and
// rows 2(w + 8j) + h of the dA partials; with 1 or 2 partitions 4 waves and
// the whole reduction per wave (measured: 8 waves are slower at V = 18, K = 1,
// 7% faster at V = 25, K = 3). Requires K * ceil(V/2) * ceil(V/32) <= 48 (B-operand
// registers) and the k_spatial_bwd4 host conditions.
constexpr int bwd5_nw(int kmax) { return kmax >= 3 ? 8 : 4; }

template <int V, int RB, int KMAX>
__global__ __launch_bounds__(bwd5_nw(KMAX) * 64) void k_spatial_bwd5(
    const float *__restrict__ H, const float *__restrict__ x, const float *__restrict__ mean,
    const float *__restrict__ invstd, const float *__restrict__ g, const float *__restrict__ b,
    const float *__restrict__ A, float *dx, float *dA, double *sd, double *sdn, int C, int T,
    int K, int64_t rows, int write_dx, int relu, PrevBn prev, float *dA_part) {
  constexpr int VH = (V + 1) / 2;           // MFMA k-steps over v
  constexpr int NW = bwd5_nw(KMAX);         // waves
  constexpr int NH = NW / 4;                // reduction halves of the dx GEMM
  constexpr int VQ = (VH + NH - 1) / NH;    // MFMA k-steps per half
  constexpr int NT = (V + 31) / 32;         // 32-column output tiles over w
  constexpr int DW = NT * 32;
  constexpr int MAXSEG = 32;
  constexpr int PL = (RB * V + 255) / 256 * 256;  // plane pitch: whole 16-byte DMA rounds
  constexpr int NRT = RB / 32;                    // 32-row tiles per block
  constexpr bool DREG = KMAX * NT * NT <= 4;      // dA accumulators resident in VGPRs
  extern __shared__ __attribute__((aligned(16))) float smem[];
  __shared__ double segv[4][MAXSEG];  // [sd | sdn | s1 | s2] per channel segment
  const int BUF = (K + 1) * PL;  // one buffer: K H planes + x plane (prev mode: U)
  float *dxs = smem + 2 * BUF;   // [RB][V]: reduction half 0, then dx
  float *dxs2 = dxs + PL;        // [RB][V]: reduction half 1 (NH == 2)
  const bool pv = prev.mean != nullptr;
  const int ns = pv ? 4 : 2;
  double *const gdst[4] = {sd, sdn, prev.s1, prev.s2};
  float *dred = dxs + NH * PL;   // [K][DW][DW]
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int hi = lane >> 5, lo = lane & 31;
  const int CT = C * T;  // rows per clip (rows < 2^31: host check)
  const int nblocks = (int)(rows / RB);
  const bool seg_lds = (RB + T - 1) / T + 1 <= MAXSEG;

  const int kh = wave >> 2, rtile = wave & 3;  // dx reduction half, row tile
  // B operand of the dx GEMM, this wave's half: Bm[k][j][t] = A_k[v = 2(kh VQ + j) + hi]
  // [w = 32t + lo] (0 outside)
  float Bm[KMAX][VQ][NT];
#pragma unroll
  for (int k = 0; k < KMAX; ++k)
#pragma unroll
    for (int s2 = 0; s2 < VQ; ++s2)
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        const int v = 2 * (kh * VQ + s2) + hi, w = 32 * t + lo;
        Bm[k][s2][t] = (k < K && v < V && w < V) ? A[(k * V + v) * V + w] : 0.f;
      }

  auto stage = [&](int blk, float *buf) {
    const int r0 = blk * RB;
    const int n0 = r0 / CT, rem0 = r0 - n0 * CT;
    constexpr int ND = PL / 256;  // DMA rounds per plane
    const __amdgpu_buffer_rsrc_t rx = make_rsrc(x + (int64_t)r0 * V, (int64_t)RB * V);
    for (int i = wave; i < ND; i += NW)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rx, buf + K * PL + i * 256, 16,
                                               (unsigned)(i * 256 + lane * 4) * 4u, 0, 0, 0);
    for (int k = 0; k < K; ++k) {
      const __amdgpu_buffer_rsrc_t rh =
          make_rsrc(H + ((int64_t)(n0 * K + k) * CT + rem0) * V, (int64_t)RB * V);
      for (int i = wave; i < ND; i += NW)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rh, buf + k * PL + i * 256, 16,
                                                 (unsigned)(i * 256 + lane * 4) * 4u, 0, 0, 0);
    }
  };

  for (int i = tid; i < K * DW * DW; i += NW * 64) dred[i] = 0.f;
  floatx16 dacc[DREG ? KMAX : 1][NT][NT];
  auto zero_dacc = [&](int kd) {
#pragma unroll
    for (int p2 = 0; p2 < NT; ++p2)
#pragma unroll
      for (int q2 = 0; q2 < NT; ++q2)
#pragma unroll
        for (int i = 0; i < 16; ++i) dacc[kd][p2][q2][i] = 0.f;
  };
#pragma unroll
  for (int kd = 0; kd < (DREG ? KMAX : 1); ++kd) zero_dacc(kd);
  // dacc[kd] -> dred[k] (LDS atomics), then zero
  auto flush_dacc = [&](int k) {
    const int kd = DREG ? k : 0;
#pragma unroll
    for (int p2 = 0; p2 < NT; ++p2)
#pragma unroll
      for (int q2 = 0; q2 < NT; ++q2)
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const int v = p2 * 32 + (i & 3) + 8 * (i >> 2) + 4 * hi;
          const int w = q2 * 32 + lo;
          if (v < V && w < V) atomicAdd(dred + (k * DW + v) * DW + w, dacc[kd][p2][q2][i]);
        }
    zero_dacc(kd);
  };
  int blk = blockIdx.x;
  if (blk < nblocks) stage(blk, smem);
  for (int it = 0; blk < nblocks; ++it, blk += gridDim.x) {
    float *buf = smem + (it & 1) * BUF;
    float *Hs = buf, *xs = buf + K * PL;
    if (tid < MAXSEG) segv[0][tid] = segv[1][tid] = segv[2][tid] = segv[3][tid] = 0.0;
    __syncthreads();  // block blk staged (vmcnt(0)); previous block fully retired
    if (blk + (int)gridDim.x < nblocks) stage(blk + gridDim.x, smem + ((it + 1) & 1) * BUF);
    const int r0 = blk * RB;
    const int n0 = r0 / CT, rem0 = r0 - n0 * CT;
    const int cfirst = n0 * C + rem0 / T;  // global (n*C + ci) of row r0
    // dx tile rtile (32 rows), reduction half kh, on MFMA (RB = 64: waves 2, 3,
    // 6, 7 idle here)
    if (rtile < NRT) {
      floatx16 acc[NT];
#pragma unroll
      for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int i = 0; i < 16; ++i) acc[t][i] = 0.f;
#pragma unroll
      for (int k = 0; k < KMAX; ++k) {
        if (k < K) {
          const float *hr = Hs + k * PL + (rtile * 32 + lo) * V + hi + 2 * kh * VQ;
#pragma unroll
          for (int s2 = 0; s2 < VQ; ++s2) {
            const float av = (2 * (kh * VQ + s2) + hi < V) ? hr[2 * s2] : 0.f;
#pragma unroll
            for (int t = 0; t < NT; ++t) acc[t] = mfma32(av, Bm[k][s2][t], acc[t]);
          }
        }
      }
#pragma unroll
      for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const int row = rtile * 32 + (i & 3) + 8 * (i >> 2) + 4 * hi;
          const int w = 32 * t + lo;
          if (w < V) (kh ? dxs2 : dxs)[row * V + w] = acc[t][i];
        }
    }
    __syncthreads();  // dx tile complete
    // per row (TPR threads each, interleaved joints): BN1 sums, BN1(x) in
    // place; per-channel-segment sums (a wave's rows usually share one
    // channel: then one wave reduction)
    {
      constexpr int TPR = NW * 64 / RB;
      const int rl = tid / TPR, part = tid % TPR;
      const int rem = rem0 + rl;
      const int ci = rem / T;
      const int seg = n0 * C + ci - cfirst;
      const float mu = mean[ci], is = invstd[ci];
      const float a = is * g[ci], be = b[ci];
      // prev mode: the staged plane is the previous block's U; its output x =
      // ReLU((U - pmu) * pa + pb) as that block's output pass formed it
      const float pmu = pv ? prev.mean[ci] : 0.f, pis = pv ? prev.invstd[ci] : 1.f;
      const float pa = pv ? pis * prev.g[ci] : 1.f, pb = pv ? prev.b[ci] : 0.f;
      float sv[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int j = 0; j < (V + TPR - 1) / TPR; ++j) {
        const int w = part + j * TPR;
        if (w < V) {
          float xv = xs[rl * V + w];
          float uh = 0.f;
          bool pm = false;
          if (pv) {
            const float t = (xv - pmu) * pa + pb;
            uh = (xv - pmu) * pis;
            pm = t > 0.f;
            xv = pm ? t : 0.f;
          }
          float d = NH == 2 ? dxs[rl * V + w] + dxs2[rl * V + w] : dxs[rl * V + w];
          const float bn = (xv - mu) * a + be;
          if (relu && bn <= 0.f) d = 0.f;  // ReLU'(BN1(x))
          dxs[rl * V + w] = d;
          sv[0] += d;
          sv[1] = fmaf(d, (xv - mu) * is, sv[1]);
          if (pm) {
            sv[2] += d;
            sv[3] = fmaf(d, uh, sv[3]);
          }
          xs[rl * V + w] = relu ? fmaxf(bn, 0.f) : bn;
        }
      }
      STGCN_ROWPASS_SUMS(sv, ns, seg, ci);
    }
    __syncthreads();  // BN1(x) rows and segment sums complete
    if (seg_lds && tid < MAXSEG) {
      const int gc = cfirst + tid;  // global (n*C + ci)
      const int rlast = r0 + RB - 1;
      const int glast = (rlast / CT) * C + (rlast % CT) / T;
      if (gc <= glast) {
        const int cc = gc % C;
        for (int i = 0; i < ns; ++i) atomicAdd(gdst[i] + cc, segv[i][tid]);
      }
    }
    // dA partials on MFMA: wave takes row pairs kk = wave + 8j; accumulators
    // stay in registers across blocks (DREG) or are flushed per block
#pragma unroll
    for (int k = 0; k < KMAX; ++k) {
      if (k < K) {
        floatx16(&dk)[NT][NT] = dacc[DREG ? k : 0];
        const float *hk = Hs + k * PL;
#pragma unroll
        for (int j = 0; j < RB / (2 * NW); ++j) {
          const int rr = 2 * (wave + NW * j) + hi;
          float av[NT], bw[NT];
#pragma unroll
          for (int t = 0; t < NT; ++t) {
            const int c = t * 32 + lo;
            av[t] = c < V ? hk[rr * V + c] : 0.f;
            bw[t] = c < V ? xs[rr * V + c] : 0.f;
          }
#pragma unroll
          for (int p2 = 0; p2 < NT; ++p2)
#pragma unroll
            for (int q2 = 0; q2 < NT; ++q2) dk[p2][q2] = mfma32(av[p2], bw[q2], dk[p2][q2]);
        }
        if (!DREG) flush_dacc(k);
      }
    }
    if (write_dx) {
      float *dst = dx + (int64_t)r0 * V;
      for (int e = tid; e < RB * V / 4; e += NW * 64)
        *reinterpret_cast<float4 *>(dst + e * 4) = *reinterpret_cast<const float4 *>(dxs + e * 4);
    }
  }
  if constexpr (DREG) {
    // the waves' register tiles into the zeroed LDS accumulator one wave after
    // the other (plain adds, one owner lane per entry): a fixed order
    __syncthreads();
    for (int wv = 0; wv < NW; ++wv) {
      if (wave == wv) {
#pragma unroll
        for (int k = 0; k < KMAX; ++k)
          if (k < K) {
#pragma unroll
            for (int p2 = 0; p2 < NT; ++p2)
#pragma unroll
              for (int q2 = 0; q2 < NT; ++q2)
#pragma unroll
                for (int i = 0; i < 16; ++i) {
                  const int v = p2 * 32 + (i & 3) + 8 * (i >> 2) + 4 * hi;
                  const int w = q2 * 32 + lo;
                  if (v < V && w < V) dred[(k * DW + v) * DW + w] += dacc[k][p2][q2][i];
                }
          }
      }
      __syncthreads();
    }
  }
  __syncthreads();
  for (int i = tid; i < K * V * V; i += NW * 64) {
    const int k = i / (V * V), rm = i - k * V * V, v = rm / V, w = rm - v * V;
    if (dA_part)  // (deterministic: launch_dA_reduce adds the partials in order)
      dA_part[(int64_t)blockIdx.x * K * V * V + i] = dred[(k * DW + v) * DW + w];
    else
      atomicAdd(dA + i, dred[(k * DW + v) * DW + w]);
  }
}

template <int V, int RB>
static size_t bwd5_lds(int K) {
  constexpr int PL = (RB * V + 255) / 256 * 256;
  constexpr int DW = (V + 31) / 32 * 32;
  const int nh = bwd5_nw(K) / 4;
  return sizeof(float) * ((size_t)(2 * (K + 1) + nh) * PL + (size_t)K * DW * DW);
}

template <int V, int RB, int KT>
static bool launch_bwd5(const float *H, const float *x, const float *mean, const float *invstd,
                        const float *g, const float *b, const float *A, float *dx, float *dA,
                        double *sd, double *sdn, int C, int T, int K, int64_t rows,
                        int write_dx, int relu, hipStream_t s, const PrevBn &prev,
                        bool dry = false, float *dA_part = nullptr, int64_t part_cap = 0,
                        int64_t *nparts = nullptr) {
  const size_t lds = bwd5_lds<V, RB>(K);
  if (lds > 160 * 1024 - 1024 || ((int64_t)C * T) % RB != 0 || rows >= (int64_t)1 << 31) return false;
  const int per_cu = std::max(1, std::min(8, (int)((160 * 1024) / (lds + 1024))));
  const dim3 grid((unsigned)std::min<int64_t>(rows / RB, 256 * per_cu));
  if (K != KT) return false;
  if (dry) return true;
  float *part = dA_part && (int64_t)grid.x <= part_cap ? dA_part : nullptr;
  if (part && nparts) *nparts = grid.x;
  hipLaunchKernelGGL((k_spatial_bwd5<V, RB, KT>), grid, dim3(bwd5_nw(KT) * 64), lds, s, H, x, mean, invstd, g,
                     b, A, dx, dA, sd, sdn, C, T, K, rows, write_dx, relu, prev, part);
  return true;
}

// k_spatial_bwd6: k_spatial_bwd5 for joint counts above 32 (two 32-column
// output tiles, V = 50: the two-person graph) with up to 3 partitions, where
// bwd5's register-resident B operand (all column tiles) and LDS dA accumulator
// do not fit. RB = 64 rows per block, 8 waves (two per SIMD, so one wave's LDS
// reads and row pass run under the other's MFMAs): dx = 2 row tiles x 2 column
// tiles x 2 halves of the joint reduction (wave = tile + 4 * half, each half
// keeping only its k-steps of its column tile of A_k as the B operand:
// K * 13 VGPRs; the halves meet in LDS, summed by the row pass); the K x 2 x 2
// dA tiles x 2 row halves of the block are dealt to the 8 waves (K each) and
// stay in registers for the whole persistent loop, flushed once by global
// atomics. Staging, BN1 sums and the dx store as in bwd5.
// exact 3-way bf16 split (x == h + m + l, see kernels_x3.hip) for bwd6's dA
typedef __bf16 bwd6_bf8 __attribute__((ext_vector_type(8)));
typedef __bf16 bwd6_bf2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ unsigned bwd6_pk(float a, float b) {
  const bwd6_bf2 v = {(__bf16)a, (__bf16)b};
  return __builtin_bit_cast(unsigned, v);
}
__device__ __forceinline__ void bwd6_split2(float a, float b, unsigned &h, unsigned &m,
                                            unsigned &l) {
  h = bwd6_pk(a, b);
  const float ra = a - __builtin_bit_cast(float, h << 16);
  const float rb = b - __builtin_bit_cast(float, h & 0xffff0000u);
  m = bwd6_pk(ra, rb);
  l = bwd6_pk(ra - __builtin_bit_cast(float, m << 16), rb - __builtin_bit_cast(float, m & 0xffff0000u));
}
__device__ __forceinline__ floatx16 bwd6_mfma(uint4 a, uint4 b, floatx16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bwd6_bf8, a),
                                                 __builtin_bit_cast(bwd6_bf8, b), c, 0, 0, 0);
}

// BF (STGCN_F_BF16 blocks): H and A to 2^-16 (h + m planes; the dropped terms
// are below 2^-16 of each product), f(BN1(x)) of the dA GEMM to bf16: three
// products for dx and two for dA instead of six each. (H to bf16 alone moved
// the residual V = 50 block's BN1 bias gradient to 4.5x the bf16 reference's
// own error, past the 3x gate.)
template <int V, int KMAX, bool BF>
__global__ __launch_bounds__(512, 1) void k_spatial_bwd6(
    const float *__restrict__ H, const float *__restrict__ x, const float *__restrict__ mean,
    const float *__restrict__ invstd, const float *__restrict__ g, const float *__restrict__ b,
    const float *__restrict__ A, float *dx, float *dA, double *sd, double *sdn, int C, int T,
    int K, int64_t rows, int write_dx, int relu, PrevBn prev, float *dA_part) {
  constexpr int RB = 64, NW = 8;
  static_assert(V > 32 && V <= 64, "two 32-column tiles");
  constexpr int MAXSEG = 32;
  constexpr int PL = (RB * V + 255) / 256 * 256;  // plane pitch: whole 16-byte DMA rounds
  extern __shared__ __attribute__((aligned(16))) float smem[];
  __shared__ double segv[4][MAXSEG];  // [sd | sdn | s1 | s2] per channel segment
  const int BUF = (K + 1) * PL;  // one buffer: K H planes + x plane (prev mode: U)
  float *dxs = smem + 2 * BUF;   // [RB][V]: reduction half 0, then dx
  float *dxs2 = dxs + PL;        // [RB][V]: reduction half 1
  const bool pv = prev.mean != nullptr;
  const int ns = pv ? 4 : 2;
  double *const gdst[4] = {sd, sdn, prev.s1, prev.s2};
  // f(BN1(x)) split into 3 bf16 planes, joint-major [w][row] (pitch XTP: 16-byte
  // row groups at an odd 16-byte stride), the dA GEMM's B operand
  constexpr int XTP = RB + 8, XTPL = V * XTP * 2;
  char *XT = reinterpret_cast<char *>(dxs2 + PL);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int hi = lane >> 5, lo = lane & 31;
  const int CT = C * T;
  const int nblocks = (int)(rows / RB);
  const bool seg_lds = (RB + T - 1) / T + 1 <= MAXSEG;
  const int rt = wave & 1, ct = (wave >> 1) & 1, kh = wave >> 2;  // this wave's dx tile, half

  // B operand of the dx GEMM (v_mfma_f32_32x32x16_bf16 on exact 3-way splits):
  // column tile ct, joints v = 32 kh + 16 ks + 8 hi + j (ks = 0, 1): this wave's
  // half of the reduction, A_k[v][w = 32ct + lo] split into h / m / l planes
  uint4 Bh[KMAX][2], Bmd[KMAX][2], Bl[KMAX][2];
#pragma unroll
  for (int k = 0; k < KMAX; ++k)
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const int v0 = 32 * kh + 16 * ks + 8 * hi, w = 32 * ct + lo;
      float bv[8];
#pragma unroll
      for (int j = 0; j < 8; ++j)
        bv[j] = (k < K && v0 + j < V && w < V) ? A[(k * V + v0 + j) * V + w] : 0.f;
      bwd6_split2(bv[0], bv[1], Bh[k][ks].x, Bmd[k][ks].x, Bl[k][ks].x);
      bwd6_split2(bv[2], bv[3], Bh[k][ks].y, Bmd[k][ks].y, Bl[k][ks].y);
      bwd6_split2(bv[4], bv[5], Bh[k][ks].z, Bmd[k][ks].z, Bl[k][ks].z);
      bwd6_split2(bv[6], bv[7], Bh[k][ks].w, Bmd[k][ks].w, Bl[k][ks].w);
    }

  auto stage = [&](int blk, float *buf) {
    const int r0 = blk * RB;
    const int n0 = r0 / CT, rem0 = r0 - n0 * CT;
    constexpr int ND = PL / 256;
    const __amdgpu_buffer_rsrc_t rx = make_rsrc(x + (int64_t)r0 * V, (int64_t)RB * V);
    for (int i = wave; i < ND; i += NW)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rx, buf + K * PL + i * 256, 16,
                                               (unsigned)(i * 256 + lane * 4) * 4u, 0, 0, 0);
    for (int k = 0; k < K; ++k) {
      const __amdgpu_buffer_rsrc_t rh =
          make_rsrc(H + ((int64_t)(n0 * K + k) * CT + rem0) * V, (int64_t)RB * V);
      for (int i = wave; i < ND; i += NW)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rh, buf + k * PL + i * 256, 16,
                                                 (unsigned)(i * 256 + lane * 4) * 4u, 0, 0, 0);
    }
  };

  // dA tiles of this wave: j = (wave & 3) + 4i (i < KMAX) -> (k = i, p2 = (j / 2) & 1,
  // q2 = j & 1), over rows kh*32..+31 of each block
  floatx16 dacc[KMAX], dacl[KMAX];
#pragma unroll
  for (int i = 0; i < KMAX; ++i)
#pragma unroll
    for (int e = 0; e < 16; ++e) dacc[i][e] = dacl[i][e] = 0.f;

  int blk = blockIdx.x;
  if (blk < nblocks) stage(blk, smem);
  for (int it = 0; blk < nblocks; ++it, blk += gridDim.x) {
    float *buf = smem + (it & 1) * BUF;
    float *Hs = buf, *xs = buf + K * PL;
    if (tid < MAXSEG) segv[0][tid] = segv[1][tid] = segv[2][tid] = segv[3][tid] = 0.0;
    __syncthreads();  // block blk staged (vmcnt(0)); previous block fully retired
    if (blk + (int)gridDim.x < nblocks) stage(blk + gridDim.x, smem + ((it + 1) & 1) * BUF);
    const int r0 = blk * RB;
    const int n0 = r0 / CT, rem0 = r0 - n0 * CT;
    const int cfirst = n0 * C + rem0 / T;
    {  // dx tile (rt, ct), reduction half kh: six bf16 products per fp32 product
      floatx16 acc, acl;
#pragma unroll
      for (int i = 0; i < 16; ++i) acc[i] = acl[i] = 0.f;
#pragma unroll
      for (int k = 0; k < KMAX; ++k) {
        if (k < K) {
#pragma unroll
          for (int ks = 0; ks < 2; ++ks) {
            const int v0 = 32 * kh + 16 * ks + 8 * hi;
            const float *hr = Hs + k * PL + (rt * 32 + lo) * V + v0;
            float av[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) av[j] = v0 + j < V ? hr[j] : 0.f;
            uint4 ah, am, al;
            bwd6_split2(av[0], av[1], ah.x, am.x, al.x);
            bwd6_split2(av[2], av[3], ah.y, am.y, al.y);
            bwd6_split2(av[4], av[5], ah.z, am.z, al.z);
            bwd6_split2(av[6], av[7], ah.w, am.w, al.w);
            acc = bwd6_mfma(ah, Bh[k][ks], acc);
            acl = bwd6_mfma(ah, Bmd[k][ks], acl);
            acl = bwd6_mfma(am, Bh[k][ks], acl);
            if constexpr (!BF) {
              acl = bwd6_mfma(ah, Bl[k][ks], acl);
              acl = bwd6_mfma(am, Bmd[k][ks], acl);
              acl = bwd6_mfma(al, Bh[k][ks], acl);
            }
          }
        }
      }
      acc += acl;
      float *dst = kh ? dxs2 : dxs;
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int row = rt * 32 + (i & 3) + 8 * (i >> 2) + 4 * hi;
        const int w = 32 * ct + lo;
        if (w < V) dst[row * V + w] = acc[i];
      }
    }
    __syncthreads();  // dx tile halves complete
    {  // per row (8 threads each): dx = sum of halves, BN1 sums, BN1(x) in place (see bwd5)
      constexpr int TPR = NW * 64 / RB;
      const int rl = tid / TPR, part = tid % TPR;
      const int rem = rem0 + rl;
      const int ci = rem / T;
      const int seg = n0 * C + ci - cfirst;
      const float mu = mean[ci], is = invstd[ci];
      const float a = is * g[ci], be = b[ci];
      const float pmu = pv ? prev.mean[ci] : 0.f, pis = pv ? prev.invstd[ci] : 1.f;
      const float pa = pv ? pis * prev.g[ci] : 1.f, pb = pv ? prev.b[ci] : 0.f;
      float sv[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int j = 0; j < (V + TPR - 1) / TPR; ++j) {
        const int w = part + j * TPR;
        if (w < V) {
          float xv = xs[rl * V + w];
          float uh = 0.f;
          bool pm = false;
          if (pv) {  // prev mode: the staged plane is the previous block's U (see bwd5)
            const float t = (xv - pmu) * pa + pb;
            uh = (xv - pmu) * pis;
            pm = t > 0.f;
            xv = pm ? t : 0.f;
          }
          float d = dxs[rl * V + w] + dxs2[rl * V + w];
          const float bn = (xv - mu) * a + be;
          if (relu && bn <= 0.f) d = 0.f;
          dxs[rl * V + w] = d;
          sv[0] += d;
          sv[1] = fmaf(d, (xv - mu) * is, sv[1]);
          if (pm) {
            sv[2] += d;
            sv[3] = fmaf(d, uh, sv[3]);
          }
          const float f = relu ? fmaxf(bn, 0.f) : bn;
          const __bf16 fh = (__bf16)f;
          __bf16 *xt = reinterpret_cast<__bf16 *>(XT) + w * XTP + rl;
          xt[0] = fh;
          if constexpr (!BF) {
            const float r1 = f - (float)fh;
            const __bf16 fm = (__bf16)r1;
            xt[XTPL / 2] = fm;
            xt[XTPL] = (__bf16)(r1 - (float)fm);
          }
        }
      }
      STGCN_ROWPASS_SUMS(sv, ns, seg, ci);
    }
    __syncthreads();  // BN1(x) rows, dx and segment sums complete
    if (seg_lds && tid < MAXSEG) {
      const int gc = cfirst + tid;
      const int rlast = r0 + RB - 1;
      const int glast = (rlast / CT) * C + (rlast % CT) / T;
      if (gc <= glast) {
        const int cc = gc % C;
        for (int i = 0; i < ns; ++i) atomicAdd(gdst[i] + cc, segv[i][tid]);
      }
    }
    // dA tiles: dA_k[v in p2][w in q2] += sum_rows H_k[row][v] f(BN1(x))[row][w],
    // rows kh*32..+31 as two 16-row k-steps of v_mfma_f32_32x32x16_bf16 on the
    // exact 3-way splits: six products, h*h apart from the five cross terms
    {
      const int p2 = (wave >> 1) & 1, q2 = wave & 1;
      const int cv = p2 * 32 + lo, cw = q2 * 32 + lo;
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        const int rb = kh * 32 + ks * 16 + 8 * hi;  // this lane's 8 rows
        uint4 bh = {0, 0, 0, 0}, bm = bh, bl = bh;
        if (cw < V) {
          const char *xt = XT + (cw * XTP + rb) * 2;
          bh = *reinterpret_cast<const uint4 *>(xt);
          if constexpr (!BF) {
            bm = *reinterpret_cast<const uint4 *>(xt + XTPL);
            bl = *reinterpret_cast<const uint4 *>(xt + 2 * XTPL);
          }
        }
#pragma unroll
        for (int i = 0; i < KMAX; ++i) {
          if (i < K) {
            const float *hk = Hs + i * PL + rb * V + cv;
            float av[8];
#pragma unroll
            for (int e = 0; e < 8; ++e) av[e] = cv < V ? hk[e * V] : 0.f;
            uint4 ah, am, al;
            bwd6_split2(av[0], av[1], ah.x, am.x, al.x);
            bwd6_split2(av[2], av[3], ah.y, am.y, al.y);
            bwd6_split2(av[4], av[5], ah.z, am.z, al.z);
            bwd6_split2(av[6], av[7], ah.w, am.w, al.w);
            dacc[i] = bwd6_mfma(ah, bh, dacc[i]);
            dacl[i] = bwd6_mfma(am, bh, dacl[i]);
            if constexpr (!BF) {
              dacl[i] = bwd6_mfma(ah, bm, dacl[i]);
              dacl[i] = bwd6_mfma(ah, bl, dacl[i]);
              dacl[i] = bwd6_mfma(am, bm, dacl[i]);
              dacl[i] = bwd6_mfma(al, bh, dacl[i]);
            }
          }
        }
      }
    }
    if (write_dx) {
      float *dst = dx + (int64_t)r0 * V;
      for (int e = tid; e < RB * V / 4; e += NW * 64)
        *reinterpret_cast<float4 *>(dst + e * 4) = *reinterpret_cast<const float4 *>(dxs + e * 4);
    }
  }
#pragma unroll
  for (int i = 0; i < KMAX; ++i) {
    const int j = (wave & 3) + 4 * i;
    const int k = j >> 2, p2 = (j >> 1) & 1, q2 = j & 1;
    if (k < K) {
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int v = p2 * 32 + (e & 3) + 8 * (e >> 2) + 4 * hi;
        const int w = q2 * 32 + lo;
        if (v < V && w < V) {
          // (deterministic: one slot per row half -- waves w, w + 4 hold the same
          // entries -- added in order by launch_dA_reduce)
          if (dA_part)
            dA_part[((int64_t)blockIdx.x * 2 + (wave >> 2)) * K * V * V + (k * V + v) * V + w] =
                dacc[i][e] + dacl[i][e];
          else
            atomicAdd(dA + (k * V + v) * V + w, dacc[i][e] + dacl[i][e]);
        }
      }
    }
  }
}

template <int V, int KT, bool BF>
static bool launch_bwd6(const float *H, const float *x, const float *mean, const float *invstd,
                        const float *g, const float *b, const float *A, float *dx, float *dA,
                        double *sd, double *sdn, int C, int T, int K, int64_t rows,
                        int write_dx, int relu, hipStream_t s, const PrevBn &prev,
                        bool dry = false, float *dA_part = nullptr, int64_t part_cap = 0,
                        int64_t *nparts = nullptr) {
  constexpr int RB = 64;
  constexpr int PL = (RB * V + 255) / 256 * 256;
  const size_t lds = sizeof(float) * ((size_t)(2 * (K + 1) + 2) * PL) + 3 * (size_t)V * (RB + 8) * 2;
  if (K != KT || lds > 160 * 1024 - 1024 || ((int64_t)C * T) % RB != 0 ||
      rows >= (int64_t)1 << 31)
    return false;
  if (dry) return true;
  const dim3 grid((unsigned)std::min<int64_t>(rows / RB, 256));
  float *part = dA_part && 2 * (int64_t)grid.x <= part_cap ? dA_part : nullptr;
  if (part && nparts) *nparts = 2 * (int64_t)grid.x;
  hipLaunchKernelGGL((k_spatial_bwd6<V, KT, BF>), grid, dim3(512), lds, s, H, x, mean, invstd, g, b,
                     A, dx, dA, sd, sdn, C, T, K, rows, write_dx, relu, prev, part);
  return true;
}

// k_gather_mfma: G_k = f(BN1(x)) A_k^T on the fp32 matrix cores (joint counts
// 25 and 50 with 3 partitions, where k_gather4's one-row-per-thread VALU
// contraction is the slow part). Persistent, x row blocks double-buffered by
// LDS-DMA; block = RB = 128 / NT rows = 4 MFMA tiles (32 rows x one 32-joint
// column tile), one per wave. A-operand: f(BN1(x))[row][w] computed once per
// block from the staged rows (per-lane row constants); B-operand: the wave's
// column tile of A_k^T (B[w][v] = A_k[v][w]) resident in VGPRs. The K output
// tiles leave through LDS as float4 stores (each partition's block of G is
// contiguous).
template <int V, int KMAX>
__global__ __launch_bounds__(256, 2) void k_gather_mfma(
    const float *__restrict__ x, const float *__restrict__ mean, const float *__restrict__ invstd,
    const float *__restrict__ g, const float *__restrict__ b, const float *__restrict__ A,
    float *G, int C, int T, int K, int64_t rows, int relu) {
  constexpr int NT = (V + 31) / 32;
  constexpr int RB = 128 / NT;
  constexpr int NRT = RB / 32;
  constexpr int VH = (V + 1) / 2;
  constexpr int PL = (RB * V + 255) / 256 * 256;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float *obuf = smem + 2 * PL;  // [K][PL]
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int hi = lane >> 5, lo = lane & 31;
  const int CT = C * T;
  const int nblocks = (int)(rows / RB);
  const int rt = wave % NRT, ct = wave / NRT;
  float Bm[KMAX][VH];
#pragma unroll
  for (int k = 0; k < KMAX; ++k)
#pragma unroll
    for (int s2 = 0; s2 < VH; ++s2) {
      const int w = 2 * s2 + hi, v = 32 * ct + lo;
      Bm[k][s2] = (k < K && v < V && w < V) ? A[(k * V + v) * V + w] : 0.f;
    }
  auto stage = [&](int blk, float *buf) {
    constexpr int ND = PL / 256;
    const __amdgpu_buffer_rsrc_t rx = make_rsrc(x + (int64_t)blk * RB * V, (int64_t)RB * V);
    for (int i = wave; i < ND; i += 4)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rx, buf + i * 256, 16,
                                               (unsigned)(i * 256 + lane * 4) * 4u, 0, 0, 0);
  };
  int blk = blockIdx.x;
  if (blk < nblocks) stage(blk, smem);
  for (int it = 0; blk < nblocks; ++it, blk += gridDim.x) {
    const float *xs = smem + (it & 1) * PL;
    __syncthreads();  // block staged; previous block's stores done with obuf
    if (blk + (int)gridDim.x < nblocks) stage(blk + gridDim.x, smem + ((it + 1) & 1) * PL);
    const int r0 = blk * RB;
    const int n0 = r0 / CT, rem0 = r0 - n0 * CT;
    const int row = rt * 32 + lo;
    const int ci = (rem0 + row) / T;
    const float mu = mean[ci], a = invstd[ci] * g[ci], be = b[ci];
    float fv[VH];
#pragma unroll
    for (int s2 = 0; s2 < VH; ++s2) {
      const int w = 2 * s2 + hi;
      const float t = w < V ? (xs[row * V + w] - mu) * a + be : 0.f;
      fv[s2] = w < V ? (relu ? fmaxf(t, 0.f) : t) : 0.f;
    }
#pragma unroll
    for (int k = 0; k < KMAX; ++k) {
      if (k < K) {
        floatx16 acc;
#pragma unroll
        for (int i = 0; i < 16; ++i) acc[i] = 0.f;
#pragma unroll
        for (int s2 = 0; s2 < VH; ++s2) acc = mfma32(fv[s2], Bm[k][s2], acc);
        float *ok = obuf + k * PL;
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const int r = rt * 32 + (i & 3) + 8 * (i >> 2) + 4 * hi;
          const int v = 32 * ct + lo;
          if (v < V) ok[r * V + v] = acc[i];
        }
      }
    }
    __syncthreads();  // output tiles complete
    for (int k = 0; k < K; ++k) {
      float *dst = G + ((int64_t)(n0 * K + k) * CT + rem0) * V;
      const float *src = obuf + k * PL;
      for (int e = tid; e < RB * V / 4; e += 256)
        *reinterpret_cast<float4 *>(dst + e * 4) = *reinterpret_cast<const float4 *>(src + e * 4);
    }
  }
}

template <int V, int KT>
static bool launch_gather_mfma(const float *x, const float *mean, const float *invstd,
                               const float *g, const float *b, const float *A, float *G, int C,
                               int T, int K, int64_t rows, int relu, hipStream_t s) {
  constexpr int NT = (V + 31) / 32;
  constexpr int RB = 128 / NT;
  constexpr int PL = (RB * V + 255) / 256 * 256;
  if (K != KT || ((int64_t)C * T) % RB != 0 || (RB * V) % 4 != 0 || rows >= (int64_t)1 << 31)
    return false;
  const size_t lds = sizeof(float) * (size_t)(2 + K) * PL;
  const int per_cu = std::max(1, std::min(2, (int)((160 * 1024) / (lds + 512))));
  const dim3 grid((unsigned)std::min<int64_t>(rows / RB, 256 * per_cu));
  hipLaunchKernelGGL((k_gather_mfma<V, KT>), grid, dim3(256), lds, s, x, mean, invstd, g, b, A, G,
                     C, T, K, rows, relu);
  return true;
}

static int bwd3_rows(int V, int K) {
  // rows per block: 256 when the per-row LDS footprint is small, else 64
  const int VP = (V + 3) & ~3;
  return (K * V + VP) * 4 * 256 <= 48 * 1024 ? 256 : 64;
}

static bool joint_fast(int V) { return V == 18 || V == 25 || V == 50; }

bool gather_prev_supported(int C, int T, int V) {
  return STGCN_AB_JOINT3 == 0 && joint_fast(V) && ((int64_t)C * T) % 256 == 0 &&
         sizeof(float) * ((size_t)2 * 256 * V + (size_t)V * ((V + 3) & ~3)) <= 160 * 1024;
}

hipError_t launch_gather_fwd(const float *x, const float *mean, const float *invstd,
                             const float *g, const float *b, const float *A, float *G, int N,
                             int C, int T, int V, int K, int relu, hipStream_t s, unsigned *amax,
                             const PrevBn *pv) {
  constexpr bool joint3 = STGCN_AB_JOINT3 != 0;  // A/B builds only (ab_switches.h)
  const PrevBn pvb = pv ? *pv : PrevBn{};
  if (pv && (K != 1 || !gather_prev_supported(C, T, V) || ((uintptr_t)x & 15) != 0 ||
             ((uintptr_t)G & 15) != 0))
    return hipErrorInvalidValue;  // (x from U: k_gather4 only; checked by the caller first)
  if (!pv && !joint3 && !amax && K > 1 && (V == 25 || V == 50) && ((uintptr_t)x & 15) == 0 &&
      ((uintptr_t)G & 15) == 0) {  // partitioned graphs: contraction on MFMA
    const int64_t rows = (int64_t)N * C * T;
    const bool done =
        V == 25 ? (launch_gather_mfma<25, 2>(x, mean, invstd, g, b, A, G, C, T, K, rows, relu, s) ||
                   launch_gather_mfma<25, 3>(x, mean, invstd, g, b, A, G, C, T, K, rows, relu, s))
                : (launch_gather_mfma<50, 2>(x, mean, invstd, g, b, A, G, C, T, K, rows, relu, s) ||
                   launch_gather_mfma<50, 3>(x, mean, invstd, g, b, A, G, C, T, K, rows, relu, s));
    if (done) return hipGetLastError();
  }
  const size_t lds4 = sizeof(float) * ((size_t)2 * 256 * V + (size_t)K * V * ((V + 3) & ~3));
  if (!joint3 && joint_fast(V) && ((int64_t)C * T) % 256 == 0 && ((uintptr_t)x & 15) == 0 &&
      ((uintptr_t)G & 15) == 0 && lds4 <= 160 * 1024) {
    const int64_t rows = (int64_t)N * C * T;
    const dim3 grid4((unsigned)(rows / 256));
    if (V == 18)
      hipLaunchKernelGGL(k_gather4<18>, grid4, dim3(256), lds4, s, x, mean, invstd, g, b, A, G, C, T, K, rows, relu, amax, pvb);
    else if (V == 25)
      hipLaunchKernelGGL(k_gather4<25>, grid4, dim3(256), lds4, s, x, mean, invstd, g, b, A, G, C, T, K, rows, relu, amax, pvb);
    else
      hipLaunchKernelGGL(k_gather4<50>, grid4, dim3(256), lds4, s, x, mean, invstd, g, b, A, G, C, T, K, rows, relu, amax, pvb);
    return hipGetLastError();
  }
  if (joint_fast(V)) {
    const int VP = (V + 3) & ~3;
    const int64_t rows = (int64_t)N * C * T;
    const size_t lds3 = sizeof(float) * (size_t)K * V * VP;
    const dim3 grid3((unsigned)((rows + 255) / 256));
    if (V == 18)
      hipLaunchKernelGGL(k_gather3<18>, grid3, dim3(256), lds3, s, x, mean, invstd, g, b, A, G, C, T, K, rows, relu, amax);
    else if (V == 25)
      hipLaunchKernelGGL(k_gather3<25>, grid3, dim3(256), lds3, s, x, mean, invstd, g, b, A, G, C, T, K, rows, relu, amax);
    else
      hipLaunchKernelGGL(k_gather3<50>, grid3, dim3(256), lds3, s, x, mean, invstd, g, b, A, G, C, T, K, rows, relu, amax);
    return hipGetLastError();
  }
  const size_t lds = sizeof(float) * ((size_t)K * V * V + kGatherTC * V);
  hipLaunchKernelGGL(k_gather_fwd, dim3((T + kGatherTC - 1) / kGatherTC, N), dim3(256), lds, s, x,
                     mean, invstd, g, b, A, G, C, T, V, K, relu, amax);
  return hipGetLastError();
}

// out[c][v] += sum_t X[n][c][t][v]   (fp64), one block per (c, n)
__global__ __launch_bounds__(256) void k_sum_nt(const float *X, int C, int T, int V,
                                                double *out) {
  __shared__ double part[256];
  const int c = blockIdx.x, n = blockIdx.y;
  const float *src = X + ((int64_t)n * C + c) * T * V;
  const int tpb = 256 / V;  // frame lanes per joint
  const int tid = threadIdx.x;
  double s = 0.0;
  if (tid < tpb * V) {
    const int v = tid % V, tt = tid / V;
    for (int t = tt; t < T; t += tpb) s += src[t * V + v];
  }
  part[tid] = s;
  __syncthreads();
  if (tid < V) {
    double acc = 0.0;
    for (int tt = 0; tt < tpb; ++tt) acc += part[tt * V + tid];
    atomicAdd(out + c * V + tid, acc);
  }
}

// k_sum_nt with float4 loads: 4*A consecutive floats per pass, A = the
// largest multiple of the float4 period of V (V / gcd(4, V)) <= 256, so each
// thread's 4 lanes keep fixed joints across passes; the per-thread fp64
// partials are then folded per joint through LDS. A row (n, c) that does not
// start on a 16-byte boundary (T * V odd or 2 mod 4) is read from the aligned
// address below its start: its elements sit `shift` floats into the float4
// stream, lanes outside [0, T*V) are masked, and the fold maps stream position
// q to joint (q - shift) mod V.
__global__ __launch_bounds__(256) void k_sum_nt4(const float *X, int C, int T, int V,
                                                 double *out) {
  __shared__ double part[1024];
  const int c = blockIdx.x, n = blockIdx.y, tid = threadIdx.x;
  const int L = T * V;
  const int per = V / (V % 4 == 0 ? 4 : (V % 2 == 0 ? 2 : 1));  // float4 period
  const int A = 256 / per * per;                                 // active threads
  const int64_t start = ((int64_t)n * C + c) * L;
  const int shift = (int)(start & 3);
  const float4 *src = reinterpret_cast<const float4 *>(X + (start - shift));
  const int nf = (L + shift + 3) / 4;
  double a0 = 0.0, a1 = 0.0, a2 = 0.0, a3 = 0.0;
  if (tid < A) {
    for (int f = tid; f < nf; f += A) {
      const float4 q = src[f];
      const int p0 = 4 * f - shift;  // row position of lane 0
      if (p0 >= 0 && p0 + 3 < L) {
        a0 += q.x;
        a1 += q.y;
        a2 += q.z;
        a3 += q.w;
      } else {
        if (p0 >= 0 && p0 < L) a0 += q.x;
        if (p0 + 1 >= 0 && p0 + 1 < L) a1 += q.y;
        if (p0 + 2 >= 0 && p0 + 2 < L) a2 += q.z;
        if (p0 + 3 >= 0 && p0 + 3 < L) a3 += q.w;
      }
    }
  }
  part[4 * tid] = a0;
  part[4 * tid + 1] = a1;
  part[4 * tid + 2] = a2;
  part[4 * tid + 3] = a3;
  __syncthreads();
  if (tid < V) {
    double acc = 0.0;
    // stream position q holds joint (q - shift) mod V; 4*A is a multiple of V
    for (int q = (tid + shift) % V; q < 4 * A; q += V) acc += part[q];
    atomicAdd(out + c * V + tid, acc);
  }
}

// k_sum_nt4 over a bf16 tensor (capi.hip dz_bf16): 4 bf16 = 8 bytes per load,
// the same period / shift bookkeeping (8-byte boundary below a row's start)
__global__ __launch_bounds__(256) void k_sum_nt4_bf16(const __bf16 *X, int C, int T, int V,
                                                      double *out) {
  __shared__ double part[1024];
  const int c = blockIdx.x, n = blockIdx.y, tid = threadIdx.x;
  const int L = T * V;
  const int per = V / (V % 4 == 0 ? 4 : (V % 2 == 0 ? 2 : 1));
  const int A = 256 / per * per;
  const int64_t start = ((int64_t)n * C + c) * L;
  const int shift = (int)(start & 3);
  const uint2 *src = reinterpret_cast<const uint2 *>(X + (start - shift));
  const int nf = (L + shift + 3) / 4;
  double a0 = 0.0, a1 = 0.0, a2 = 0.0, a3 = 0.0;
  auto f0 = [](unsigned w) { return __builtin_bit_cast(float, w << 16); };
  auto f1 = [](unsigned w) { return __builtin_bit_cast(float, w & 0xffff0000u); };
  if (tid < A) {
    for (int f = tid; f < nf; f += A) {
      const uint2 q = src[f];
      const int p0 = 4 * f - shift;
      if (p0 >= 0 && p0 < L) a0 += f0(q.x);
      if (p0 + 1 >= 0 && p0 + 1 < L) a1 += f1(q.x);
      if (p0 + 2 >= 0 && p0 + 2 < L) a2 += f0(q.y);
      if (p0 + 3 >= 0 && p0 + 3 < L) a3 += f1(q.y);
    }
  }
  part[4 * tid] = a0;
  part[4 * tid + 1] = a1;
  part[4 * tid + 2] = a2;
  part[4 * tid + 3] = a3;
  __syncthreads();
  if (tid < V) {
    double acc = 0.0;
    for (int q = (tid + shift) % V; q < 4 * A; q += V) acc += part[q];
    atomicAdd(out + c * V + tid, acc);
  }
}

hipError_t launch_sum_nt(const float *X, int N, int C, int T, int V, double *out, hipStream_t s,
                         int x_bf16) {
  if (x_bf16) {  // (a bf16 tensor in an fp32-sized, 16-byte aligned buffer)
    if (V > 256 || ((int64_t)N * C * T * V) % 4 != 0) return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_sum_nt4_bf16, dim3(C, N), dim3(256), 0, s,
                       reinterpret_cast<const __bf16 *>(X), C, T, V, out);
    return hipGetLastError();
  }
  // (rows of any alignment: the float4 kernel reads from the 16-byte boundary
  // below a row's start; X 16-byte aligned and a whole number of float4 in
  // total, so no read passes the tensor's end)
  if (((uintptr_t)X & 15) == 0 && ((int64_t)N * C * T * V) % 4 == 0 && V <= 256) {
    hipLaunchKernelGGL(k_sum_nt4, dim3(C, N), dim3(256), 0, s, X, C, T, V, out);
    return hipGetLastError();
  }
  hipLaunchKernelGGL(k_sum_nt, dim3(C, N), dim3(256), 0, s, X, C, T, V, out);
  return hipGetLastError();
}

// dbW[k*R+co] = sum_v SdZ[co][v] * rowsum(A_k)[v]
// dA[k][v][w]  = sum_co bW[k*R+co] * SdZ[co][v]      (bias part of dA; all w)
// One block per partition k; V <= 90 (K*V*V <= 8192, checked by the C-ABI).
__global__ __launch_bounds__(256) void k_spatial_small(const double *SdZ, const float *A,
                                                       const float *bW, int K, int R, int V,
                                                       float *dbW, float *dA) {
  __shared__ double rs[128], part[256];
  const int k = blockIdx.x, tid = threadIdx.x;
  for (int v = tid; v < V; v += 256) {
    double ra = 0.0;
    for (int w = 0; w < V; ++w) ra += A[((int64_t)k * V + v) * V + w];
    rs[v] = ra;
  }
  __syncthreads();
  for (int co = tid; co < R; co += 256) {
    double acc = 0.0;
    for (int v = 0; v < V; ++v) acc += SdZ[co * V + v] * rs[v];
    dbW[k * R + co] = (float)acc;
  }
  // bias part of dA: thread (v, j) sums co = j, j + P, ... (P = 256 / V parts)
  const int P = 256 / V;
  const int v = tid % V, j = tid / V;
  double acc = 0.0;
  if (j < P)
    for (int co = j; co < R; co += P) acc += (double)bW[k * R + co] * SdZ[co * V + v];
  part[tid] = acc;
  __syncthreads();
  if (tid < V) {
    double t = 0.0;
    for (int jj = 0; jj < P; ++jj) t += part[jj * V + tid];
    rs[tid] = t;  // rowsums no longer needed
  }
  __syncthreads();
  for (int i = tid; i < V * V; i += 256) dA[(int64_t)k * V * V + i] = (float)rs[i / V];
}

hipError_t launch_spatial_small(const double *SdZ, const float *A, const float *bW, int K, int R,
                                int V, float *dbW, float *dA, hipStream_t s) {
  if (V > 128) return hipErrorInvalidValue;
  hipLaunchKernelGGL(k_spatial_small, dim3(K), dim3(256), 0, s, SdZ, A, bW, K, R, V, dbW, dA);
  return hipGetLastError();
}

constexpr int kDxTC = 16;  // frames per spatial-dx block

// Per (n, frame chunk), looping over input channels ci:
//   dxhat[t][w] = sum_k sum_v H[k*C+ci][t][v] * A[k][v][w]     (-> dx buffer)
//   dA[k][v][w] += sum_t H[k*C+ci][t][v] * BN1(x)[ci][t][w]     (LDS accumulator)
//   sd[ci] += sum dxhat, sdn[ci] += sum dxhat * xnorm          (BN1 backward)
__global__ __launch_bounds__(256) void k_spatial_dx(const float *H, const float *x,
                                                    const float *mean, const float *invstd,
                                                    const float *g, const float *b,
                                                    const float *A, float *dx, float *dA,
                                                    double *sd, double *sdn, int C, int T, int V,
                                                    int K, int write_dx, int relu) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  __shared__ double red[8];
  const int KVV = K * V * V;
  float *As = smem;             // [K][V][V]
  float *dAs = As + KVV;        // [K][V][V] block-local dA
  float *xb = dAs + KVV;        // [TC][V] BN1 output
  float *Hs = xb + kDxTC * V;   // [K][TC][V]
  const int n = blockIdx.y, t0 = blockIdx.x * kDxTC;
  int tc = T - t0;
  if (tc > kDxTC) tc = kDxTC;
  const int tid = threadIdx.x;
  for (int i = tid; i < KVV; i += 256) {
    As[i] = A[i];
    dAs[i] = 0.f;
  }
  const int L = T * V;
  for (int ci = 0; ci < C; ++ci) {
    __syncthreads();
    const int64_t xo = ((int64_t)n * C + ci) * L + (int64_t)t0 * V;
    const float mu = mean[ci], is = invstd[ci], a = is * g[ci], be = b[ci];
    for (int i = tid; i < tc * V; i += 256) {
      const float t = (x[xo + i] - mu) * a + be;
      xb[i] = relu ? fmaxf(t, 0.f) : t;
    }
    for (int i = tid; i < K * tc * V; i += 256) {
      const int k = i / (tc * V), rem = i - k * tc * V;
      Hs[k * kDxTC * V + rem] = H[(((int64_t)n * K + k) * C + ci) * L + (int64_t)t0 * V + rem];
    }
    __syncthreads();
    // dxhat and BN1 partial sums
    double s = 0.0, sn = 0.0;
    for (int o = tid; o < tc * V; o += 256) {
      const int t = o / V, w = o - t * V;
      float acc = 0.f;
      for (int k = 0; k < K; ++k) {
        const float *hr = Hs + (k * kDxTC + t) * V;
        const float *ac = As + k * V * V + w;
        for (int v = 0; v < V; ++v) acc = fmaf(hr[v], ac[v * V], acc);
      }
      const float xn = (x[xo + o] - mu) * is;
      if (relu && (x[xo + o] - mu) * a + be <= 0.f) acc = 0.f;  // ReLU'(BN1(x))
      if (write_dx) dx[xo + o] = acc;
      s += acc;
      sn += (double)acc * xn;
    }
    // dA partials: each thread owns entries e = tid + 256*j
    for (int e = tid; e < KVV; e += 256) {
      const int k = e / (V * V), rem = e - k * V * V;
      const int v = rem / V, w = rem - v * V;
      float acc = dAs[e];
      for (int t = 0; t < tc; ++t) acc = fmaf(Hs[(k * kDxTC + t) * V + v], xb[t * V + w], acc);
      dAs[e] = acc;
    }
    block_sum2_atomic<256>(s, sn, sd + ci, sdn + ci, red);
  }
  for (int e = tid; e < KVV; e += 256) atomicAdd(dA + e, dAs[e]);
}

// the bwd5 / bwd6 launch (or, dry, whether one of them takes this shape)
static bool launch_bwd56(const float *H, const float *x, const float *mean, const float *invstd,
                         const float *g, const float *b, const float *A, float *dx, float *dA,
                         double *sd, double *sdn, int N, int C, int T, int V, int K, int write_dx,
                         int relu, bool bf6, hipStream_t s, const PrevBn &prev, bool dry,
                         float *dA_part = nullptr, int64_t part_cap = 0,
                         int64_t *nparts = nullptr) {
  constexpr bool joint3 = STGCN_AB_JOINT3 != 0;  // A/B builds only (ab_switches.h)
  const bool aligned = ((int64_t)N * C * T * V) % 4 == 0 && ((uintptr_t)x & 15) == 0 &&
                       ((uintptr_t)H & 15) == 0 && ((uintptr_t)dx & 15) == 0;
  if (!joint3 && aligned && K <= 3 && K * ((V + 1) / 2) * ((V + 31) / 32) <= 48) {
    const int64_t rows = (int64_t)N * C * T;
    bool done = false;
#define STGCN_BWD5(VV, RR, KK)                                                              \
  launch_bwd5<VV, RR, KK>(H, x, mean, invstd, g, b, A, dx, dA, sd, sdn, C, T, K, rows, write_dx, \
                          relu, s, prev, dry, dA_part, part_cap, nparts)
    // partitions K: 1 (uniform), 2 (distance), 3 (spatial) labelling
    if (V == 18)
      done = STGCN_BWD5(18, 128, 1) || STGCN_BWD5(18, 64, 1) || STGCN_BWD5(18, 128, 2) ||
             STGCN_BWD5(18, 64, 2) || STGCN_BWD5(18, 128, 3) || STGCN_BWD5(18, 64, 3);
    else if (V == 25)
      done = STGCN_BWD5(25, 128, 1) || STGCN_BWD5(25, 64, 1) || STGCN_BWD5(25, 128, 2) ||
             STGCN_BWD5(25, 64, 2) || STGCN_BWD5(25, 128, 3) || STGCN_BWD5(25, 64, 3);
    else if (V == 50)
      done = STGCN_BWD5(50, 64, 1) || STGCN_BWD5(50, 64, 2) || STGCN_BWD5(50, 64, 3);
#undef STGCN_BWD5
    if (done) return true;
  }
  if (!joint3 && aligned && V == 50 && K <= 3) {  // two-person graph, 2 or 3 partitions
    const int64_t rows = (int64_t)N * C * T;
    bool done = false;
#define STGCN_BWD6(KK, BF)                                                                     \
  launch_bwd6<50, KK, BF>(H, x, mean, invstd, g, b, A, dx, dA, sd, sdn, C, T, K, rows, write_dx, \
                          relu, s, prev, dry, dA_part, part_cap, nparts)
    if (bf6)
      done = STGCN_BWD6(1, true) || STGCN_BWD6(2, true) || STGCN_BWD6(3, true);
    else
      done = STGCN_BWD6(1, false) || STGCN_BWD6(2, false) || STGCN_BWD6(3, false);
#undef STGCN_BWD6
    if (done) return true;
  }
  return false;
}

bool spatial_dx_prev_supported(int N, int C, int T, int V, int K) {
  // (16-byte aligned operands: any non-null aligned stand-in pointer)
  const float *p = reinterpret_cast<const float *>(uintptr_t(256));
  return launch_bwd56(p, p, nullptr, nullptr, nullptr, nullptr, nullptr, const_cast<float *>(p),
                      nullptr, nullptr, nullptr, N, C, T, V, K, 1, 0, true, nullptr, PrevBn(), true);
}

hipError_t launch_spatial_dx(const float *H, const float *x, const float *mean,
                             const float *invstd, const float *g, const float *b, const float *A,
                             float *dx, float *dA, double *sd, double *sdn, int N, int C, int T,
                             int V, int K, int write_dx, int relu, int bf16ops, hipStream_t s,
                             const PrevBn *prev, float *dA_part, int64_t part_cap,
                             int64_t *nparts) {
  if (nparts) *nparts = 0;
  // (STGCN_AB_BWD6_EXACT: the exact-split k_spatial_bwd6 for bf16 blocks too)
  constexpr bool exact6 = STGCN_AB_BWD6_EXACT != 0;
  const bool bf6 = bf16ops && !exact6;
  const PrevBn pv = prev ? *prev : PrevBn();
  if (launch_bwd56(H, x, mean, invstd, g, b, A, dx, dA, sd, sdn, N, C, T, V, K, write_dx, relu,
                   bf6, s, pv, false, dA_part, part_cap, nparts))
    return hipGetLastError();
  if (pv.mean) return hipErrorInvalidValue;  // (callers check spatial_dx_prev_supported)
  if (joint_fast(V) && K <= 3) {
    const int VP = (V + 3) & ~3;
    const int RB = bwd3_rows(V, K);
    const int64_t rows = (int64_t)N * C * T;
    const int DW3 = (V + 31) / 32 * 32;
    const size_t lds3 = sizeof(float) * ((size_t)K * V * VP + (size_t)K * RB * V + (size_t)RB * VP +
                                         (size_t)(RB / 64) * K * DW3 * DW3);
    const dim3 grid3((unsigned)((rows + RB - 1) / RB));
    // (per-workgroup dA partials where the caller's buffer holds them all)
    float *part = dA_part && (int64_t)grid3.x <= part_cap ? dA_part : nullptr;
    if (part && nparts) *nparts = grid3.x;
    if (V == 18)
      hipLaunchKernelGGL(k_spatial_bwd3<18>, grid3, dim3(RB), lds3, s, H, x, mean, invstd, g, b, A,
                         dx, dA, sd, sdn, C, T, K, rows, write_dx, relu, part);
    else if (V == 25)
      hipLaunchKernelGGL(k_spatial_bwd3<25>, grid3, dim3(RB), lds3, s, H, x, mean, invstd, g, b, A,
                         dx, dA, sd, sdn, C, T, K, rows, write_dx, relu, part);
    else
      hipLaunchKernelGGL(k_spatial_bwd3<50>, grid3, dim3(RB), lds3, s, H, x, mean, invstd, g, b, A,
                         dx, dA, sd, sdn, C, T, K, rows, write_dx, relu, part);
    return hipGetLastError();
  }
  if (K * V * V > 8192) return hipErrorInvalidValue;
  const size_t lds = sizeof(float) * (2 * (size_t)K * V * V + kDxTC * V + (size_t)K * kDxTC * V);
  hipLaunchKernelGGL(k_spatial_dx, dim3((T + kDxTC - 1) / kDxTC, N), dim3(256), lds, s, H, x,
                     mean, invstd, g, b, A, dx, dA, sd, sdn, C, T, V, K, write_dx, relu);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// Deterministic dA (the spatial backward's per-workgroup partials, dA_part):
// pass 1 sums the partials of chunk y in a fixed order (four interleaved fp64
// chains per entry, combined in order) into lvl[y][e]; pass 2 adds
// sum_y lvl[y][e] (in y order, fp64) to dA[e]. Replaces the fp32 atomics whose
// arrival order made dA differ from run to run at the 1e-3 level on this
// heavily cancelling gradient.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_dA_reduce1(const float *__restrict__ part, int64_t nparts,
                                                    int n, int64_t chunk, double *lvl) {
  __shared__ double sm[4][64];
  const int t = threadIdx.x & 63, g = threadIdx.x >> 6;
  const int e = blockIdx.x * 64 + t;
  const int64_t p0 = (int64_t)blockIdx.y * chunk, p1 = min(nparts, p0 + chunk);
  double s = 0.0;
  if (e < n) {
    int64_t q = p0 + g;
    for (; q + 12 < p1; q += 16) {  // (four loads in flight)
      const float a0 = part[q * n + e], a1 = part[(q + 4) * n + e];
      const float a2 = part[(q + 8) * n + e], a3 = part[(q + 12) * n + e];
      s += a0;
      s += a1;
      s += a2;
      s += a3;
    }
    for (; q < p1; q += 4) s += part[q * n + e];
  }
  sm[g][t] = s;
  __syncthreads();
  if (g == 0 && e < n) lvl[(int64_t)blockIdx.y * n + e] = ((sm[0][t] + sm[1][t]) + sm[2][t]) + sm[3][t];
}

__global__ __launch_bounds__(256) void k_dA_reduce2(const double *__restrict__ lvl, int ny, int n,
                                                    float *dA) {
  // (four groups of 64 lanes, each over every fourth level with all its loads
  // in flight, combined in group order)
  __shared__ double sm[4][64];
  const int t = threadIdx.x & 63, g = threadIdx.x >> 6;
  const int e = blockIdx.x * 64 + t;
  double s = 0.0;
  if (e < n) {
#pragma unroll
    for (int i = 0; i < kDaLvl / 4; ++i) {
      const int y = g + 4 * i;
      if (y < ny) s += lvl[(int64_t)y * n + e];
    }
  }
  sm[g][t] = s;
  __syncthreads();
  if (g == 0 && e < n)
    dA[e] = (float)((double)dA[e] + (((sm[0][t] + sm[1][t]) + sm[2][t]) + sm[3][t]));
}

hipError_t launch_dA_reduce(const float *part, int64_t nparts, int n, double *lvl, float *dA,
                            hipStream_t s) {
  if (nparts <= 0) return hipSuccess;
  if (!part || !lvl || !dA || n <= 0) return hipErrorInvalidValue;
  const int ny = (int)std::min<int64_t>(kDaLvl, nparts);
  const int64_t chunk = (nparts + ny - 1) / ny;
  const int nb = (n + 63) / 64;
  hipLaunchKernelGGL(k_dA_reduce1, dim3(nb, ny), dim3(256), 0, s, part, nparts, n, chunk, lvl);
  hipLaunchKernelGGL(k_dA_reduce2, dim3(nb), dim3(256), 0, s, lvl, ny, n, dA);
  return hipGetLastError();
}

}  // namespace stgcn
