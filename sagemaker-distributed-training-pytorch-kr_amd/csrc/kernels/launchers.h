// C ABI of the gfx950 kernel library. Kernel translation units (.hip) are compiled without any
// PyTorch headers (fast, torch-independent builds); `bindings.cpp` is the only file that sees
// ATen and forwards tensors + the current HIP stream to these launchers.
//
// dtype codes: 0 = fp32, 1 = bf16, 2 = fp16.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

extern "C" {

// layernorm.hip
int smdt_ln_bwd_nblocks(int64_t rows, int H);
hipError_t smdt_layernorm_fwd(int dtype, int wdtype, const void* x, const void* res,
                              const void* bias, const void* gamma, const void* beta, void* y,
                              void* s_out, float* mean, float* rstd, int64_t rows, int H,
                              float eps, float p_drop, uint64_t seed, uint64_t offset, int rms,
                              const void* x2, hipStream_t st);
hipError_t smdt_layernorm_bwd(int dtype, int wdtype, const void* dy, const void* ds_in,
                              const void* s, const void* gamma, const float* mean,
                              const float* rstd, void* ds_out, void* dx_out, float* partials,
                              int nblocks, float* dgamma, float* dbeta, float* dbias,
                              int64_t rows, int H, float p_drop, uint64_t seed, uint64_t offset,
                              int rms, int acc_mask, const void* dy2, hipStream_t st);

// bias_act.hip
int smdt_bias_act_slices(int64_t rows, int N);
hipError_t smdt_bias_act_fwd(int dtype, int act, const void* x, const void* bias, void* y,
                             int64_t rows, int N, hipStream_t st);
hipError_t smdt_bias_act_bwd(int dtype, int act, const void* dy, const void* x, const void* bias,
                             void* dx, float* partials, float* dbias, int64_t rows, int N,
                             int accumulate, hipStream_t st);
hipError_t smdt_col_sum(const float* partials, int nslices, int N, float* out, int accumulate,
                        hipStream_t st);
// column sums of dy [rows, N] into out[N] (fp32; accumulate = add into out)
hipError_t smdt_bias_grad(int dtype, const void* dy, int64_t rows, int N, float* partials,
                          float* out, int accumulate, hipStream_t st);
hipError_t smdt_swiglu_fwd(int dtype, const void* x, void* y, int64_t rows, int F,
                           hipStream_t st);
hipError_t smdt_swiglu_bwd(int dtype, const void* dy, const void* x, void* dx, int64_t rows,
                           int F, hipStream_t st);

// softmax.hip
hipError_t smdt_softmax_fwd(int dtype, int mode, const void* x, const uint8_t* mask, void* y,
                            int64_t rows, int sq, int sk, int heads, float scale,
                            hipStream_t st);
hipError_t smdt_softmax_bwd(int dtype, int mode, const void* dy, const void* y, void* dx,
                            int64_t rows, int sq, int sk, float scale, hipStream_t st);

// graph-safe dropout RNG (flash_attn.hip): the device step counter every dropout kernel mixes into
// its key at run time (null: none). Set by the bindings (set_rng_step), read by the launchers.
extern "C" void smdt_set_rng_step(uint32_t* counter);
extern "C" uint32_t* smdt_rng_step();

// optim.hip
hipError_t smdt_adam(float* master, const float* grad, float* m, float* v, void* model_out,
                     int model_dtype, int64_t n, float lr, float beta1, float beta2, float eps,
                     float wd, float bc1, float bc2, int adamw, const float* grad_mul,
                     const int* found_inf, const float* hyper, hipStream_t st);
int smdt_sumsq_nblocks(int64_t n);
hipError_t smdt_sumsq(int dtype, const void* x, int64_t n, float* partial, int nblocks,
                      float* out, int* found_inf, hipStream_t st);
hipError_t smdt_clip_coef(const float* sumsq, float max_norm, float inv_scale, float* mul_out,
                          float* norm_out, hipStream_t st);
hipError_t smdt_scale(int dtype, void* x, int64_t n, const float* mul, float cmul,
                      hipStream_t st);
hipError_t smdt_cast(int in_dtype, int out_dtype, const void* x, void* y, int64_t n,
                     int accumulate, hipStream_t st);

// rope.hip
hipError_t smdt_rope(int dtype, void* x, int64_t ntok, int nh, int64_t tok_stride,
                     int64_t head_stride, int rot, const float* cos_t, const float* sin_t,
                     int pos_div, int pos_mod, int backward, hipStream_t st);

// transpose.hip
hipError_t smdt_transpose16(const void* in, void* out, int64_t R, int64_t C, hipStream_t st);
// link_standin.hip: paced copy standing in for a TP-pair exchange in single-GPU rank emulation
hipError_t smdt_paced_copy(const void* src, void* dst, int64_t nbytes, int blocks, int64_t ns, hipStream_t st);
// dst[r] = map[r] >= 0 ? src[map[r]] : 0 (rows of row_bytes, a multiple of 16)
hipError_t smdt_gather_rows(const void* src, const int64_t* map, void* dst, int64_t nrows, int64_t nsrc,
                            int64_t row_bytes, hipStream_t st);

// cross_entropy.hip
hipError_t smdt_ce_stats(int dtype, const void* logits, const int64_t* target, int64_t rows,
                         int V, int Vvalid, int64_t vstart, float* row_max, float* row_sumexp,
                         float* row_tgt, hipStream_t st);
hipError_t smdt_ce_bwd(int dtype, const void* logits, const int64_t* target, const float* gmax,
                       const float* gsum, const float* dloss, void* dlogits, int64_t rows, int V,
                       int Vvalid, int64_t vstart, int64_t ignore_index, hipStream_t st);
hipError_t smdt_ce_fused(int dtype, void* logits, const int64_t* target, float* loss, int64_t rows,
                         int V, int Vvalid, int64_t ignore_index, int local, int64_t vstart, hipStream_t st);

// augment.hip: per-sample depthwise filter (KS in {3, 5, 7}) and 3 x 3 median, fp32 NCHW
hipError_t smdt_aug_depthwise(const float* x, const float* k, float* y, int N, int C, int H, int W, int ks,
                              hipStream_t st);
hipError_t smdt_aug_median3(const float* x, float* y, int planes, int H, int W, hipStream_t st);

// flash_attn.hip
hipError_t smdt_flash_fwd(int dtype, const void* q, const void* k, const void* v, void* o,
                          float* lse, int B, int H, int Hkv, int S, int D, int64_t q_sb,
                          int64_t q_ss, int64_t q_sh, int64_t k_sb, int64_t k_ss, int64_t k_sh,
                          int64_t v_sb, int64_t v_ss, int64_t v_sh, int64_t o_sb, int64_t o_ss,
                          int64_t o_sh, float scale, int causal, float dropout_p, uint64_t seed,
                          uint64_t offset, hipStream_t st);
// delta: fp32 scratch of 2 x B x H x S (the backward's prepared per-query row constants).
hipError_t smdt_flash_bwd(int dtype, const void* q, const void* k, const void* v, const void* o,
                          const void* dout, const float* lse, float* delta, void* dq, void* dk,
                          void* dv, int B, int H, int Hkv, int S, int D, const int64_t* strides,
                          float scale, int causal, float dropout_p, uint64_t seed,
                          uint64_t offset, hipStream_t st);

// gemm_tn.hip: C[M, N] = A[M, K] . B[N, K]^T (16-bit in / out, fp32 accumulate) with an epilogue:
// epi 0 none, 1 + bias[n], 2 C = pre-activation and C2 = gelu_tanh(C + bias[n]) (bias_gelu fusion),
// 3 C = product * gelu_tanh'(aux + bias[n]) (fc2 dgrad + GeLU backward; aux = pre-activation [M, N]).
// max_blocks <= 0: one persistent workgroup per CU.
int smdt_gemm_tn_supported(int64_t M, int64_t N, int64_t K);
hipError_t smdt_gemm_tn(int dtype, int epi, const void* a, const void* b, void* c, void* c2, const void* bias,
                        const void* aux, int64_t M, int64_t N, int64_t K, int max_blocks, hipStream_t st);
// diagnostic ablations of the same kernel (benchmarks only): var bits as gemm_tn_kernel's VAR
hipError_t smdt_gemm_tn_var(int dtype, int epi, const void* a, const void* b, void* c, void* c2, const void* bias,
                            const void* aux, int64_t M, int64_t N, int64_t K, int max_blocks, int var,
                            hipStream_t st);

// wgrad_gemm.hip: main_grad[N, K] (fp32) += dy[M, N]^T . x[M, K] (bf16, or fp16 with dtype 2)
int smdt_wgrad_supported(int64_t M, int64_t N, int64_t K);
hipError_t smdt_wgrad_accumulate_t(int dtype, const void* dy, const void* x, float* main_grad, int64_t M,
                                   int64_t N, int64_t K, int max_splits, hipStream_t st);
hipError_t smdt_wgrad_accumulate(const void* dy, const void* x, float* main_grad, int64_t M, int64_t N,
                                 int64_t K, int max_splits, hipStream_t st);
struct SmdtWgradProblem {
  const void* dy;      // [M, N] bf16
  const void* x;       // [M, K] bf16
  float* main_grad;    // [N, K] fp32, += dy^T x
  int64_t M, N, K;
  float* bias_grad;    // [N] fp32, += column sums of dy (the linear's bias gradient), or null
  int overwrite;       // 1: main_grad holds no data yet — write dy^T x instead of adding (no read)
};
// Many independent wgrad accumulations in one launch per 32 (no split-K, no atomics). The
// main_grad targets of one call must not overlap.
hipError_t smdt_wgrad_grouped(const SmdtWgradProblem* probs, int n, hipStream_t st);
hipError_t smdt_wgrad_grouped_t(int dtype, const SmdtWgradProblem* probs, int n, hipStream_t st);
// the same with the tail split sized for `cus` concurrently usable CUs (0: 256, the whole chip)
hipError_t smdt_wgrad_grouped_cus(int dtype, const SmdtWgradProblem* probs, int n, int cus, hipStream_t st);

// xgmi_allreduce.hip: single-node all-reduce over HIP-IPC-mapped peer buffers.
int smdt_ar_max_ranks();
int smdt_ar_max_blocks();
int64_t smdt_ar_signal_bytes();
int smdt_ipc_handle_bytes();
hipError_t smdt_ipc_malloc(int64_t bytes, int uncached, void** ptr);  // zero-filled
hipError_t smdt_ipc_free(void* ptr);
hipError_t smdt_ipc_get_handle(void* ptr, void* handle_out);
hipError_t smdt_ipc_open(const void* handle, void** ptr);
hipError_t smdt_ipc_close(void* ptr);
hipError_t smdt_ar_read_error(void* sig, int* err);
int64_t smdt_ar_word_offset(int which);
// out = scale * sum over ranks of in (n elements, n * esize % 16 == 0). data_ptrs / sig_ptrs: the
// world ranks' staging (4 x region_bytes) and signal buffers. nranks_local > 1 = loopback: ranks
// rank .. rank + nranks_local - 1 in one launch, in/out strided by io_stride elements per rank.
// `blocks` is fixed per engine (every call of one engine must pass the same value).
hipError_t smdt_xgmi_allreduce(int dtype, const void* in, void* out, int64_t io_stride, int64_t n, float scale,
                               void* const* data_ptrs, void* const* sig_ptrs, int world, int rank,
                               int nranks_local, int64_t region_bytes, int two_shot, int blocks,
                               hipStream_t st);
// General form (xgmi_allreduce.hip header): mode 0 one-shot / 1 two-shot all-reduce, 2 reduce-scatter,
// 3 all-gather; in/out_rank_stride: loopback rows (elements).
hipError_t smdt_xgmi_collective(int mode, int dtype, const void* in, void* out, int64_t in_rank_stride,
                                int64_t out_rank_stride, int64_t n, int64_t slice_stride, float scale,
                                void* const* data_ptrs, void* const* sig_ptrs, int world, int rank, int nranks_local,
                                int64_t region_bytes, int blocks, hipStream_t st);

// xgmi_relay.hip: pairwise exchange of a TP pair routed over every xGMI link of the node (direct
// parts + relay parts staged in the other GPUs' buffers). stage_ptrs: world x (world x 2 x slot_bytes)
// staging buffers; partners[r] = r's TP partner; epoch = engine call counter (>= 1, same on both
// partners). n elements (n * esize % 16 == 0, 2 * ceil(n / world) vectors <= slot).
int64_t smdt_relay_signal_bytes();
int smdt_relay_max_sub();
hipError_t smdt_relay_read_error(void* sig, int* err);
int64_t smdt_relay_word_offset(int which);
hipError_t smdt_xgmi_relay(int dtype, const void* in, void* out, int64_t in_rank_stride, int64_t out_rank_stride,
                           int64_t n, void* const* stage_ptrs, void* const* sig_ptrs, const int* partners, int world,
                           int rank, int nranks_local, int64_t slot_bytes, int sub, uint32_t epoch, int dev_epoch,
                           hipStream_t st);
// zero one signal buffer's flags and device epoch (all ranks synchronised, no call in flight)
hipError_t smdt_relay_reset(void* sig, hipStream_t st);
// device epochs: advance the call counter of local ranks [rank, rank + nranks_local) by n
hipError_t smdt_relay_epoch_bump(void* const* sig_ptrs, int world, int rank, int nranks_local, uint32_t n,
                                 hipStream_t st);

}  // extern "C"
