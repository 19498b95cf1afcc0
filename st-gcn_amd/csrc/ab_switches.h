// Compile-time A/B alternates of the tuned kernel paths.
//
// The shipped library (build.py default) has exactly one path per
// configuration: every switch below is at its default (0, except
// STGCN_AB_F16X2_DGRAD = 1: the folded data gradient on the fp16 splits under
// STGCN_F_F16X2). A measurement build flips one with
// a -D define (`build.py`: build(variant="name", defines=("STGCN_AB_UNFUSED_SP=1",)),
// loaded as lib/libstgcn_hip_<variant>.so by scripts/), so no environment
// variable can route the product library to an untested kernel.
#pragma once

#ifndef STGCN_AB_UNFUSED_SP     // the unfused gather + W' GEMM instead of k_sp_fwd_*
#define STGCN_AB_UNFUSED_SP 0
#endif
#ifndef STGCN_AB_UNFUSED_SPB    // the H GEMM + k_spatial_bwd5/6 pair instead of k_sp_bwd_fused
#define STGCN_AB_UNFUSED_SPB 0
#endif
#ifndef STGCN_AB_SPB_X3         // k_sp_bwd_fused on exact splits for the fp32 path (cfg2)
#define STGCN_AB_SPB_X3 0
#endif
#ifndef STGCN_AB_WSP_F32        // the fp32-MFMA spatial dW' on STGCN_F_F32X3 blocks
#define STGCN_AB_WSP_F32 0
#endif
#ifndef STGCN_AB_WSP_RING       // k_wgrad_sp<.., X3> with the LDS-DMA ring
#define STGCN_AB_WSP_RING 0
#endif
#ifndef STGCN_AB_ACT_FP32       // fp32 storage of Z / dU on the bf16 path
#define STGCN_AB_ACT_FP32 0
#endif
#ifndef STGCN_AB_SLICE          // the unfused spatial backward in Infinity-Cache-sized clip slices
#define STGCN_AB_SLICE 0
#endif
#ifndef STGCN_AB_DZ_BF16        // bf16 storage of dZ on the bf16 path (capi.hip dz_bf16)
#define STGCN_AB_DZ_BF16 0
#endif
#ifndef STGCN_AB_X3_MR1         // 64-row tiles only in k_conv_x3
#define STGCN_AB_X3_MR1 0
#endif
#ifndef STGCN_AB_OLD_BF16CONV   // k_conv_bf16 for the 9/5/4-tap bf16 GEMMs
#define STGCN_AB_OLD_BF16CONV 0
#endif
#ifndef STGCN_AB_GK_SLOTS2      // two-slot staging in k_wgrad_gemm_gk
#define STGCN_AB_GK_SLOTS2 0
#endif
#ifndef STGCN_AB_SPF_NARROW25   // the 64-row k_sp_fwd_bf16 for V = 25, K = 3
#define STGCN_AB_SPF_NARROW25 0
#endif
#ifndef STGCN_AB_GENERIC_CONV   // the runtime-geometry conv kernels for every V
#define STGCN_AB_GENERIC_CONV 0
#endif
#ifndef STGCN_AB_JOINT3         // k_spatial_bwd3 / gather3 instead of the MFMA joint kernels
#define STGCN_AB_JOINT3 0
#endif
#ifndef STGCN_AB_WG_REGSTAGE    // register staging in k_wgrad_bf16 for bf16 P / Q at even V
#define STGCN_AB_WG_REGSTAGE 0
#endif
#ifndef STGCN_AB_S2_ACT_FP32     // fp32 Z / dU on stride-2 bf16 blocks at even V
#define STGCN_AB_S2_ACT_FP32 0
#endif
#ifndef STGCN_AB_NO_FOLD        // the unfolded spatial GEMMs on the fp32 split path (capi.hip fold_w)
#define STGCN_AB_NO_FOLD 0
#endif
#ifndef STGCN_AB_SUM_NT         // sum_{n,t} dZ by a pass over dZ on unfolded blocks
#define STGCN_AB_SUM_NT 0
#endif
#ifndef STGCN_AB_BWD6_EXACT     // exact-split k_spatial_bwd6 for bf16 blocks
#define STGCN_AB_BWD6_EXACT 0
#endif
#ifndef STGCN_AB_SPB_PAIR        // the folded block's H stored + k_spatial_bwd5 (no fused epilogue)
#define STGCN_AB_SPB_PAIR 0
#endif
#ifndef STGCN_AB_X3_NOW4        // the 8-wave 128-row k_conv_x3 for the fp16-split stride-1 forward
#define STGCN_AB_X3_NOW4 0
#endif
#ifndef STGCN_AB_F16X2_DGRAD     // 0: the folded data gradient on 3-way bf16 splits under STGCN_F_F16X2
#define STGCN_AB_F16X2_DGRAD 1
#endif
