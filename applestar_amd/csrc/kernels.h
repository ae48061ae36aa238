// Host-side launch entry points of the applestar_amd HIP kernels (gfx950).
// Every launcher takes raw device pointers + an explicit hipStream_t so it can be captured into a
// hipGraph; none allocates or synchronises.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace as {

// dtype codes shared with the bindings
enum DType : int { DT_F32 = 0, DT_BF16 = 1 };
// source dtypes of raw observation fields
enum SrcType : int { SRC_U8 = 0, SRC_I8 = 1, SRC_I16 = 2, SRC_I32 = 3, SRC_I64 = 4, SRC_F16 = 5, SRC_F32 = 6 };
enum FieldKind : int { FIELD_ONE_HOT = 0, FIELD_BINARY = 1, FIELD_SCALAR = 2 };

constexpr int kMaxFields = 40;
// Kernel-argument table describing the per-entity observation fields (passed by value).
struct EntityFields {
  const void* ptr[kMaxFields];
  int dtype[kMaxFields];
  int kind[kMaxFields];
  int offset[kMaxFields];
  int width[kMaxFields];
  int n;
};

// ---- layernorm.hip -------------------------------------------------------------------------
// y = act(LN(x + residual) * w + b); saves per-row mean/rstd and (if residual) the fp32 sum.
void layer_norm_fwd(const void* x, int x_dt, const void* res, int res_dt, const float* w, const float* b,
                    void* y, int y_dt, float* xsum, float* mean, float* rstd, long rows, int cols, float eps,
                    int act, hipStream_t s);
// dx (fp32 or bf16) and per-block partial dw/db [nblk, cols] (reduced by layer_norm_bwd_reduce).  msrc / dxm
// (optional, fp32): dxm = dx masked by (msrc > 0), for an x that is a ReLU output.
void layer_norm_bwd(const void* dy, int dy_dt, const void* xin, int xin_dt, const void* y, int y_dt,
                    const float* w, const float* mean, const float* rstd, void* dx, int dx_dt,
                    float* dw_part, float* db_part, long rows, int cols, int act, int nblk, hipStream_t s,
                    const float* msrc = nullptr, float* dxm = nullptr);
void column_reduce(const float* part, float* out, int nrows, int cols, hipStream_t s);
// entity packing tables (valid [B][N], packed -> padded row flat[total], segment seg[total], offsets cu[B + 1])
void entity_pack(const void* num, bool num64, int B, int N, long total, bool* valid, int64_t* flat, int64_t* seg,
                 int* cu, hipStream_t s);
// scalar-encoder embedding + ReLU (idt: 0 int64, 1 int32, 2 int16, 3 uint8, 4 int8; index clamped to [0, V))
void embed_relu_fwd(const void* table, int dt, const void* idx, int idt, void* out, long U, int V, int D,
                    hipStream_t s);
void embed_relu_bwd(const void* dout, const void* out, int dt, const void* idx, int idt, float* dtab, long U, int V,
                    int D, bool direct, hipStream_t s);
// nrows <= 1024 only (one pass, no atomics): bf16 output
void column_reduce_bf16(const float* part, void* out, int nrows, int cols, hipStream_t s);
int layer_norm_bwd_blocks(long rows);

// ---- scan.hip --------------------------------------------------------------------------------
// y[t] = a[t] * y[t+1] + b[t], t = T-1..0, y[T] = init; tensors [K, T, B] fp32 (K independent).
void reverse_scan(const float* a, const float* b, const float* init, float* y, int K, int T, int B,
                  hipStream_t s);

// ---- elementwise.hip -------------------------------------------------------------------------
// out = relu(tanh(y * sigmoid(g)) * sp + x)
void gated_residual_fwd(const void* y, const void* g, const float* sp, const void* x, const void* post, void* out,
                        int dt, long n, hipStream_t s);
// value-encoder spatial input: relu(W [sc(8) | own | enemy] + b) per NHWC pixel, one-pass backward
int vsp_in_channels();
int vsp_out_channels();
void vsp_fwd(const void* sc, const void* own, const void* enemy, const float* w, const float* b, void* out, long P,
             hipStream_t s, int dt = DT_BF16);
int vsp_bwd_blocks(long P);
// pooled (even H, W): relu(projection) -> max_pool2x2; pooled [B*H/2*W/2, 16] bf16 + argmax bytes (maxpool2
// format); backward from the pooled gradient: dSc [P, 8] (zero off the argmax pixels) and partial dW / db rows
void vsp_pool_fwd(const void* sc, const void* own, const void* enemy, const float* w, const float* b, void* pooled,
                  uint8_t* pos, int B, int H, int W, hipStream_t s, int dt = DT_BF16);
void vsp_pool_bwd(const void* dpooled, const uint8_t* pos, const void* pooled, const void* sc, const void* own,
                  const void* enemy, const float* w, void* dsc, float* part, int B, int H, int W, int nblk,
                  hipStream_t s, int dt = DT_BF16);
void vsp_bwd(const void* dout, const void* out, const void* sc, const void* own, const void* enemy, const float* w,
             void* dsc, float* part, long P, int nblk, hipStream_t s, int dt = DT_BF16);
// location-head input: relu(y0 + W_p relu(p)) per NHWC pixel and its one-pass backward (locin.hip)
bool loc_in_supported(int C, int P);
void loc_in_fwd(const void* y0, const void* p, const float* wp, void* out, long npix, int HW, hipStream_t s);
int loc_in_bwd_blocks(long npix);
void loc_in_bwd(const void* dy, const void* y, const void* p, const float* wp, void* dym, void* dp, float* part,
                long npix, int HW, int nblk, hipStream_t s);
void gated_residual_bwd(const void* dout, const void* y, const void* g, const float* sp, const void* out,
                        const void* xin, int dt, void* dy, void* dg, void* dx, float* dsp_part, long n, int nblk,
                        hipStream_t s);
int elementwise_blocks(long n);

// ---- lstm.hip --------------------------------------------------------------------------------
// LayerNorm-LSTM recurrence for H in {384, 32}. xp [T,B,4H] = LN_i(x W_ih^T); wT = W_hh^T [H][4H]
// (fp32 or bf16). Saves what BPTT needs: c_all [T+1,B,H], xhat_h/gates [T,B,4H], xhat_c [T,B,H],
// rstd_h/rstd_c [T,B].
bool lnlstm_supported(int H);
// Split recurrence (H = 384): 8 workgroups per row exchange partial products through `slab`
// ([2, Bp, 8, 4H] fwd / [2, Bp, 8, H] bwd {epoch, fp32} granules, Bp = B rounded up to 8, ZEROED before
// every launch); a poll that times out sets *err.  All Bp * 8 workgroups must be co-resident (callers
// keep B <= 16).
struct LstmSplit {
  unsigned long long* slab;
  int* err;
};
void lnlstm_fwd(const float* xp, const float* h0, const float* c0, const void* wT, int w_dt, const float* lnh_w,
                const float* lnh_b, const float* lnc_w, const float* lnc_b, int T, int B, int H, float eps, float* out,
                float* c_all, float* xhat_h, float* rstd_h, float* gates, float* xhat_c, float* rstd_c, float* hT,
                float* cT, hipStream_t s, const LstmSplit* split = nullptr, unsigned short* out_bf16 = nullptr);
// w = W_hh [4H][H]. Outputs d(xp) [T,B,4H], d(h W_hh^T) [T,B,4H], dL/d(LN_c out) [T,B,H], dh0, dc0.
void lnlstm_bwd(const float* dout, const float* dhT, const float* dcT, const float* gates, const float* c_all,
                const float* xhat_c, const float* rstd_c, const float* xhat_h, const float* rstd_h, const void* w,
                int w_dt, const float* lnh_w, const float* lnc_w, int T, int B, int H, float* dgates, float* dhg,
                float* dc_ln, float* dh0, float* dc0, hipStream_t s, const LstmSplit* split = nullptr);

// ---- entity.hip ------------------------------------------------------------------------------
// out[t] = relu(bias + sum_fields W^T[row(field value)]) for packed entity t (source row index[t]).
void entity_embed_fwd(const EntityFields& f, const int64_t* index, const void* wT, int w_dt, const float* bias,
                      void* out, int out_dt, long T, hipStream_t s);
// dW partials of the embedding from dpre = dout * [out > 0] (dout / out [T][256], dt): part
// [nchunk][256 * K_in + 256] (dW row-major | db), reduced over chunks by column_reduce; K_in <= 1024
int entity_wgrad_chunks(long T);
void entity_embed_wgrad(const EntityFields& f, const int64_t* index, const void* dout, const void* out, int dt,
                        float* part, long T, int K_in, int nchunk, hipStream_t s);
// X[t, :] = 997-wide sparse encoding of entity t (X must be zeroed).
void entity_onehot(const EntityFields& f, const int64_t* index, void* X, int x_dt, long T, int K_in, hipStream_t s);

// ---- spatial.hip -----------------------------------------------------------------------------
struct SpatialPlanes {
  const uint8_t* height;     // [B*H*W]
  const uint8_t* plane[6];   // visibility, creep, player_relative, alerts, pathable, buildable
  const int16_t* effect[6];  // [B*L] flat pixel indices (0-padded)
};
// NHWC bilinear x2 (align_corners=False); C % 4 == 0
void upsample2x_fwd(const void* x, void* y, int dt, int B, int H, int W, int C, hipStream_t s);
void upsample2x_bwd(const void* dy, void* dx, int dt, int B, int H, int W, int C, hipStream_t s,
                    const void* mask = nullptr);
// bits [B*H*W] (zeroed, size % 4 == 0): bit e set where effect e has a point
void spatial_effect_bits(const SpatialPlanes& sp, uint8_t* bits, int B, int L, int HW, hipStream_t s);
// pre [npix][32] = bias + Wd . dense(pixel);  Wd [32][24]
void spatial_dense(const SpatialPlanes& sp, const uint8_t* bits, const float* wd, const float* bias, float* pre, long npix,
                   hipStream_t s);
void spatial_dense_input(const SpatialPlanes& sp, const uint8_t* bits, void* X, int x_dt, long npix, hipStream_t s);
// pre[b, y*W+x, :] += rows[b, n, :] (32 channels) for n < entity_num[b]; and its transpose (gather)
void scatter_add_rows(const void* rows, int dt, const uint8_t* ex, const uint8_t* ey, const int64_t* entity_num,
                      float* pre, int B, int N, int H, int W, hipStream_t s);
// gate (nullable): ReLU output; dpre is then treated as dout * [gate > 0]
void gather_rows(const void* dpre, const void* gate, int dt, const uint8_t* ex, const uint8_t* ey,
                 const int64_t* entity_num, void* drows, int B, int N, int H, int W, hipStream_t s);
void relu_cast(const float* x, void* y, int dt, long n, hipStream_t s);
// fused: out [B,H,W,32] = relu(bias + Wd . dense(pixel) + sum of the rows of entities at the pixel)
void spatial_embed_fused(const SpatialPlanes& sp, const float* wd, const float* bias, const void* rows, int rows_dt,
                         const uint8_t* ex, const uint8_t* ey, const int64_t* entity_num, void* out, int out_dt, int B,
                         int N, int H, int W, int L, hipStream_t s);
// pooled: relu(embed) -> max_pool2x2 in one pass (pixel-row pairs per workgroup); pooled [B,H/2,W/2,32] bf16,
// pos [B,H/2,W/2,32] argmax bytes (maxpool2 format); needs spatial_pool_supported(H, W)
bool spatial_pool_supported(int H, int W);
void spatial_embed_pool(const SpatialPlanes& sp, const float* wd, const float* bias, const void* rows, const uint8_t* ex,
                        const uint8_t* ey, const int64_t* entity_num, void* pooled, uint8_t* pos, int B, int N, int H,
                        int W, int L, hipStream_t s, bool f32 = false);
// per-workgroup partial rows [spatial_wgrad_blocks(B)][32*24 + 32] of dWd (n-major) and db from dpre [B*H*W, 32]
int spatial_wgrad_blocks(int B);
void spatial_dense_wgrad(const SpatialPlanes& sp, const void* dpre, const void* gate, int dt, float* part, int B, int H,
                         int W, int L, hipStream_t s);
// pooled form (the fused embed + max-pool stage's backward, fp32): dpre from the pooled gradient dy, the pooled ReLU
// output y and the per-channel argmax pos ([B, H/2, W/2, 32] each) on the fly
void spatial_dense_wgrad_pooled(const SpatialPlanes& sp, const float* dy, const float* y, const uint8_t* pos,
                                float* part, int B, int H, int W, int L, hipStream_t s);
void gather_rows_pooled(const float* dy, const float* y, const uint8_t* pos, const uint8_t* ex, const uint8_t* ey,
                        const int64_t* entity_num, float* drows, int B, int N, int H, int W, hipStream_t s);

// ---- attention.hip ---------------------------------------------------------------------------
// Packed varlen MHA, head dim 128, bf16. qkv [T][3][H][128], cu [S+1] int32, out [T][H][128],
// lse2 [H][T] (log2 domain).  Backward writes dqkv [T][3][H][128]; delta scratch [H][T].
void varlen_attn_fwd(const void* qkv, const int* cu, void* out, float* lse2, int S, int max_len, int H, long Ttot,
                     float scale, hipStream_t s);
void varlen_attn_bwd(const void* qkv, const void* out, const void* dout, const float* lse2, const int* cu, void* dqkv,
                     float* delta, int S, int max_len, int H, long Ttot, float scale, hipStream_t s);
// The same in fp32 (f32-input MFMA): qkv / out / dout / dqkv fp32 - the fp32 learner step's attention.
void varlen_attn_fwd_f32(const float* qkv, const int* cu, float* out, float* lse2, int S, int max_len, int H, long Ttot,
                         float scale, hipStream_t s);
// fp32 attention split-path variant (attention_f32.hip); v < 0 only reads it.  Returns the previous value.
int attn_f32_variant(int v);
void varlen_attn_bwd_f32(const float* qkv, const float* out, const float* dout, const float* lse2, const int* cu,
                         float* dqkv, float* delta, int S, int max_len, int H, long Ttot, float scale, hipStream_t s);

}  // namespace as

namespace as {
// ---- pointer.hip -----------------------------------------------------------------------------
// Persistent selected-units sampler: one workgroup per batch row runs every pointer step on-chip.
// key [B, key_bstride/32, 32] (f32|bf16), c0 [B,256] = Wq1 ae0 + bq1, u [B,max_steps] uniforms,
// wf [256,256] bf16 = Wq1 We2, bf [256] = Wq1 be2.  Outputs: logits [B,max_steps,n1_stride] (rows
// after a row's end are left untouched), results/logp [B,max_steps], su_num [B], emb [B,32] (mean of
// selected keys, for the final autoregressive embedding), extra [B,n1_stride] (if extra_units).
void su_sample(const void* key, int key_dt, long key_bstride, const float* c0, const float* u, const int64_t* entity_num,
               const uint8_t* su_mask, const uint16_t* wf, const float* bf, const float* wq2, const float* bq2,
               const float* wih, const float* whh, const float* lni_w, const float* lni_b, const float* lnh_w,
               const float* lnh_b, const float* lnc_w, const float* lnc_b, const float* we1, const float* be1,
               float inv_temp, float eps, int B, int n1_stride, int max_steps, int extra_units, float* logits,
               int64_t* results, float* logp, int64_t* su_num, float* emb, float* extra, hipStream_t s);
}  // namespace as

namespace as {
// ---- gather.hip --------------------------------------------------------------------------------
// seg [nseg, 3] int64 = (src byte offset in arena, dst byte offset in out, byte count)
void segment_copy(const uint8_t* arena, uint8_t* out, const int64_t* seg, long nseg, hipStream_t s);
void conv_wt(const uint16_t* w, uint16_t* out, int cout, int cin, long s0, long s1, long s2, long s3,
             hipStream_t s);
}  // namespace as

namespace as {
// ---- upconv.hip --------------------------------------------------------------------------------
// y [B, 2Hl, 2Wl] fp32 = conv3x3(upsample_bilinear_x2(x), w[32,3,3]) + bias; x NHWC [B,Hl,Wl,32]
int upconv1_channels();
long upconv1_tiles(int B, int Hl, int Wl);
void upconv1_fwd(const void* x, int x_dt, const float* w, const float* bias, float* y, int B, int Hl, int Wl,
                 hipStream_t s);
// dx NHWC (x's dtype), dwb [289] = (dW[32*9], db); part [upconv1_tiles, 289] scratch
void upconv1_bwd(const void* x, int x_dt, const float* w, const float* dy, void* dx, float* part, float* dwb, int B,
                 int Hl, int Wl, hipStream_t s, bool relu_mask = false);
}  // namespace as

namespace as {
// ---- pool_reduce.hip ---------------------------------------------------------------------------
// NHWC 2x2/stride-2 max-pool; pos [B,H/2,W/2,C] uint8 window position; C % 8 == 0
void maxpool2_fwd(const void* x, void* y, uint8_t* pos, int dt, int B, int H, int W, int C, hipStream_t s);
void maxpool2_bwd(const void* dy, const uint8_t* pos, void* dx, int dt, int B, int H, int W, int C, hipStream_t s,
                  const void* mask = nullptr);
// bf16, even H / W: dx = dy at the argmax where the pooled ReLU output y > 0, else 0 (relu -> maxpool2 backward)
void maxpool2_bwd_relu(const void* dy, const uint8_t* pos, const void* y, void* dx, int B, int H, int W, int C,
                       hipStream_t s, bool f32 = false);
// out [S, C] fp32 = per-segment row sums of x [T, C] (segments cu[s]..cu[s+1]); C <= 1024, C % 4 == 0
void segment_sum(const void* x, int dt, const int* cu, float* out, int S, int C, hipStream_t s);
// mean over valid rows of x [B,N,C] (bf16 / fp32, fp32 accumulation) / max(num[b], 1) -> out [B,C] in x's dtype
void entity_mean_pool(const void* x, int dt, const bool* valid, const void* num, bool num64, void* out, int B, int N,
                      int C, hipStream_t s);
// LayerNorm affine gradients: per row slice s of ln_affine_slices(R), part[s] = [sum dy*xh (C) | sum dy (C)]
// (fp32 [R, C] inputs); reduce the slices with column_reduce when there are several
int ln_affine_slices(long R);
void ln_affine_grads(const float* dy, const float* xh, float* part, long R, int C, hipStream_t s);
// out [V, D] fp32 (zeroed) += src rows grouped by idx (V * D <= 16384)
void table_grad(const void* src, int dt, const int64_t* idx, float* out, long U, int V, int D, hipStream_t s);

// ---- conv3x3.hip -------------------------------------------------------------------------------
// out NHWC [B,H,W,Cout] bf16 = act(conv3x3_pad1(x NHWC bf16, w [Cout][3][3][Cin] bf16) + bias + res)
bool conv3x3_supported(int Cin, int Cout);
void conv3x3_fwd(const void* x, const void* w, const float* bias, const void* res, void* out, int B, int H, int W,
                 int Cin, int Cout, int act, hipStream_t s);

// ---- conv3x3_f32.hip / wgrad_f32.hip: the fp32 learner step's convolutions and weight gradients (f32 MFMA) --
bool conv3x3_f32_supported(int Cin, int Cout);
void conv3x3_f32_fwd(const float* x, const float* w, const float* bias, const float* res, float* out, int B, int H,
                     int W, int Cin, int Cout, int act, hipStream_t s);
// input-gradient conv with out = conv(x) + res + (rows < res2_rows: res2) masked by (mask > 0) (split ring kernel)
bool conv3x3_f32_epi2_supported(int Cin, int Cout);
void conv3x3_f32_fwd_epi2(const float* x, const float* w, const float* res, const float* res2, long res2_rows,
                          const float* mask, float* out, int B, int H, int W, int Cin, int Cout, hipStream_t s);
int wgrad_f32_splits(long R, int N, int K);
// out [M, N] = epi(A [M, K] . B [N, K]^T): + bias[n]; res added, or (act == ACT_DRELU) a mask res > 0; ReLU
// fp32 product mode of the f32 kernels: 0 = exact-f32 MFMA, 1 = bf16x6 split MFMA (split_mfma.h), split once at
// LDS staging (default), 2 = the same split done per wave after an fp32 LDS read (A/B reference);
// APPLESTAR_F32_MFMA=exact / regsplit select 0 / 2
void set_f32_pipe_variant(int v);   // gemm_f32 split-mode tile / ring variant (A/B switch)
int f32_conv_variant();             // conv3x3_f32 split-mode tile variant (A/B switch)
void set_f32_conv_variant(int v);
int f32_mfma_mode();
void set_f32_mfma_mode(int mode);
// few-row products of any shape (gemm_small.hip), fp32 (split / exact per f32_mfma_mode) or bf16:
//   small_nt: out [M, N] = epi(mask(A) [M, K] . B [N, K]^T); epi: + bias (fp32) (+ res | DRELU mask by res), act
//             RELU / SIGMOID; mask(A) = A * act'(amask) for mask_mode RELU / SIGMOID (amask: the layer output y)
//   small_tn: dW [N, K] = mask(dY)^T . X over R rows (dY [R, N], X [R, K]), db [N] = column sums of mask(dY)
void small_nt(const void* a, const void* b, const float* bias, const void* res, const void* amask, int mask_mode,
              void* out, long M, int N, int K, int act, bool bf16, hipStream_t s);
// split-K form for few tiles and a long K (> 4096): S slices write fp32 partial tiles part [S, M, N], then one
// pass sums them in slice order with the bias / act epilogue; small_nt_splits: S (1 = use small_nt)
int small_nt_splits(long M, int N, int K);
void small_nt_splitk(const void* a, const void* b, const float* bias, float* part, int S, void* out, long M, int N,
                     int K, int act, bool bf16, hipStream_t s);
void small_tn(const void* dy, const void* x, const void* ymask, int mask_mode, void* dw, void* db, long R, int N,
              int K, bool bf16_in, bool bf16_out, hipStream_t s);
// few-row bf16 GEMM (gemm_f32.hip): out [M, N] bf16 = epi(A [M, K] . B [N, K]^T), bf16 A / B / res, fp32 bias; K % 8 == 0
void gemm_bf16_small(const void* a, const void* b, const float* bias, const void* res, void* out, long M, int N, int K,
                     int act, hipStream_t s);
// fewer than 128 tiles of 128 x 64: the few-row kernels (gemm_f32_small / gemm_bf16_small) take the product
bool gemm_f32_is_small(long M, int N);
// bf16 GEMM (gemm_bf16.hip): out [M, N] bf16 = epi(A [M, K] . B [N, K]^T), bf16 A / B / res, fp32 bias; K % 8 == 0;
// LDS-DMA ring (f32_pipe.h, bf16 form), or gemm_bf16_small for few tiles
void gemm_bf16(const void* a, const void* b, const float* bias, const void* res, void* out, long M, int N, int K,
               int act, hipStream_t s);
void gemm_f32(const float* a, const float* b, const float* bias, const float* res, float* out, long M, int N, int K,
              int act, hipStream_t s);
// slice s writes dW at part + s * part_stride ([N][K]) and db at db_part + s * part_stride ([N])
void wgrad_f32(const float* dy, const float* x, float* dw_part, float* db_part, long part_stride, long R, int N, int K,
               int H, int W, int Cin, int S, hipStream_t st);

// ---- heads.hip: fused sampling tails of the action heads (inference) -----------------------------------
void head_sample(const void* logits, int logits_dt, long ld_logits, int B, int C, float inv_t, const uint8_t* mask,
                 long mask_ld, const int64_t* lens, const float* u, const void* table, int table_dt,
                 const float* tbias, int D, float* out_logits, int64_t* action, float* emb, hipStream_t s);
void target_unit_sample(const void* e, int e_dt, const float* w1, const float* b1, const float* w2, const float* b2,
                        const void* key, int key_dt, int B, int N, const int64_t* lens, float inv_t, const float* u,
                        float* out_logits, int64_t* action, hipStream_t s);

// ---- optim.hip: fused pytorch_norm / momentum_norm clip + Adam over a (tensor, offset) chunk table -------
int fused_adam_chunk();
// table: per tensor {p, g, m, v, numel, first chunk} (int64 x 6); chunks: per chunk {tensor, offset} (int64 x 2).
// mom / scale (fp32 [ntensors]) non-null: momentum_norm clip with threshold max_norm; else pytorch_norm at
// max_norm (0 = no clip).  hp (fp32 [3] = lr / bc1, 1 / sqrt(bc2), wd) non-null overrides those arguments.
void fused_clip_adam(const void* table, const long* chunks, int nchunks, int ntensors, float* part,
                     const float* gate, float* norm_out, float max_norm, float* mom, float* scale, float* mom_init,
                     const float* hp, float lr_bc1, float b1, float b2, float inv_sqrt_bc2, float eps, float wd,
                     int decoupled, hipStream_t s);

// ---- wgrad.hip ---------------------------------------------------------------------------------
// dw_part [S, N, K] / db_part [S, N] fp32 partials of dW = dY^T X(r, k), db = sum_r dY; dy [R, N] bf16.
// Cin == 0: x [R, K] bf16 (dense).  Cin > 0: x NHWC [R / (H W), H, W, Cin] bf16, K = 9 Cin (3x3 pad-1 conv).
// N % 8 == 0, K % 8 == 0 (Cin % 8 == 0), R * max(N, K or Cin) * 2 < 2^31.
int wgrad_splits(long R, int N, int K);

// ---- multi_copy.hip ----------------------------------------------------------------------------
constexpr int kCopyMaxT = 64;
constexpr long kCopyChunk = 8192;
constexpr long kCopyRawChunk = 16384;  // bytes per workgroup in raw mode (a multiple of 16 x 256)
struct CopyArgs {                     // passed by value (< 2 KB of kernel arguments)
  int ntensors;
  int chunk_start[kCopyMaxT + 1];     // prefix sums of ceil(n / kCopyChunk) (raw: ceil(n / kCopyRawChunk))
  const void* src[kCopyMaxT];
  void* dst[kCopyMaxT];
  long n[kCopyMaxT];                  // elements (raw: bytes)
  unsigned char dts[kCopyMaxT];       // bit 0: src fp32, bit 1: dst fp32 (else bf16), bit 2: raw bytes, same dtype,
                                      // bit 3 / 4: src uint8 / int16 (converting copies)
};
void multi_copy(const CopyArgs& a, hipStream_t s);

// Column-block assembly over a shared row count (fp32): output piece p is rows x width[p] columns of dst[p] (row
// pitch dld[p], first column doff[p]) = the sum of nsrc[p] (1..3) column blocks of the sources (pitch sld, first
// column soff).  Forward: the scalar encoder's three concatenations (embedded / context / baseline) of its module
// outputs in one launch; backward: each module's gradient as the sum of its slices of the three gradients.
constexpr int kColMaxP = 32;
struct ColSumArgs {                    // passed by value (~3 KB of kernel arguments)
  int npieces;
  long rows;
  int block_start[kColMaxP + 1];       // prefix sums of the pieces' workgroup counts
  float* dst[kColMaxP];
  int dld[kColMaxP], doff[kColMaxP], width[kColMaxP], nsrc[kColMaxP];
  const float* src[kColMaxP][3];
  int sld[kColMaxP][3], soff[kColMaxP][3];
};
void col_sum(const ColSumArgs& a, hipStream_t s);

// log-probability of the taken action for several heads in one launch (actor inference): head h has rows[h] rows
// of cols[h] logits (fp32 or bf16: bf16[h]) and an int64 action per row; out[h][r] = logit[a] - logsumexp(row)
constexpr int kLogpMaxH = 8;
struct LogpArgs {
  int nheads;
  long row_start[kLogpMaxH + 1];       // prefix sums of rows (one wave per row)
  const void* logits[kLogpMaxH];
  const int64_t* action[kLogpMaxH];
  float* out[kLogpMaxH];
  int cols[kLogpMaxH];
  unsigned char bf16[kLogpMaxH];
  long blk_start[kLogpMaxH + 1];       // set by multi_logp: first workgroup of each head
  unsigned char big[kLogpMaxH];        // set by multi_logp: a whole workgroup per row (wide rows)
};
void multi_logp(const LogpArgs& a, hipStream_t s);

// fp32 GEMM with the weight operand pre-split into bf16 fragment planes (gemm_f32_psb.hip): presplit_b builds the
// planes of B [N, K] (presplit_b_bytes(N, K) bytes), gemm_f32_psb runs out = act(A B^T + bias (+ res)) on them
long presplit_b_bytes(int N, int K);
void presplit_b(const float* b, int N, int K, bool trans, void* out, hipStream_t s);
bool gemm_f32_psb_supported(long M, int N, int K);
constexpr int kPresplitMax = 48;
struct PresplitArgs {                    // passed by value (~1.6 KB of kernel arguments)
  int n;
  int block_start[kPresplitMax + 1];
  const float* src[kPresplitMax];
  void* dst[kPresplitMax];
  int N[kPresplitMax], K[kPresplitMax];
  unsigned char trans[kPresplitMax];
};
void multi_presplit(const PresplitArgs& a, hipStream_t s);
void gemm_f32_psb(const float* a, const void* bsplit, const float* bias, const float* res, float* out, long M, int N,
                  int K, int act, int variant, hipStream_t s);
// 3 x 3 conv on the pre-split planes of w [Cout, 3, 3, Cin] (presplit_b of its [Cout, 9 Cin] view); res2 / mask:
// the input-gradient epilogue extras of conv3x3_f32_fwd_epi2 (nullptr: off)
bool conv3x3_f32_psb_supported(long M, int Cin, int Cout);
void conv3x3_f32_psb(const float* x, const void* wsplit, const float* bias, const float* res, const float* res2,
                     long res2_rows, const float* mask, float* out, int B, int H, int W, int Cin, int Cout, int act,
                     hipStream_t s);
// the same product with both operands staged through the LDS ring (conv3x3_f32_v2.hip; same support predicate)
void conv3x3_f32_v2(const float* x, const void* wsplit, const float* bias, const float* res, const float* res2,
                    long res2_rows, const float* mask, float* out, int B, int H, int W, int Cin, int Cout, int act,
                    int variant, hipStream_t s);
void gemm_f32_v2(const float* a, const void* bsplit, const float* bias, const float* res, float* out, long M, int N,
                 int K, int act, int variant, hipStream_t s);

// Strided multi-tensor copy (+ dtype conversion) into contiguous destinations: dst[t][i] for the dst index
// i = ((i0 * size1 + i1) * size2 + i2) * size3 + i3 reads src[t][base + sum_k ik * stride_k] (strides may be
// negative: flipped conv weights).  Rebuilds every derived weight form (fp32 biases, transposed GEMM weights,
// flipped/transposed conv weights) after an optimizer step in one launch per kSCopyMaxT tensors.
constexpr int kSCopyMaxT = 24;
struct StridedCopyArgs {                 // passed by value (~2.1 KB of kernel arguments)
  int ntensors;
  int chunk_start[kSCopyMaxT + 1];
  const void* src[kSCopyMaxT];
  void* dst[kSCopyMaxT];
  int n[kSCopyMaxT];
  int size[kSCopyMaxT][4];
  long stride[kSCopyMaxT][4];
  long base[kSCopyMaxT];
  unsigned char dts[kSCopyMaxT];         // bit 0: src fp32, bit 1: dst fp32 (else bf16), bit 2: tiled transpose
};
void multi_strided_copy(const StridedCopyArgs& a, hipStream_t s);

// ---- pointwise.hip -----------------------------------------------------------------------------
// y [P, cout] bf16 = act(x [P, cin] bf16 . w^T (fp32 [cout, cin]) + bias); cin, cout in {8, 16, 32}
bool pointwise_supported(int cin, int cout);
void pointwise_conv(const void* x, const float* w, const float* bias, void* y, long P, int cin, int cout, int act,
                    hipStream_t s);

// ---- act_grad.hip ------------------------------------------------------------------------------
// dpre NHWC bf16 [B, HW, C] = dout * (out > 0) (relu) or dout; dout fp32/bf16, NHWC or (dout_nchw) NCHW
// contiguous; out NHWC bf16.  C % 8 == 0 (NHWC) / C % 32 == 0 (NCHW).
void act_grad_nhwc(const void* dout, int dt, bool dout_nchw, const void* out, void* dpre, int B, int C, int HW, int relu,
                   hipStream_t s);
// partial slice s of dW at dw_part + s * part_stride, of db at db_part + s * part_stride
// out_bf16 with S == 1: dw_part / db_part are bf16 buffers receiving the final gradient (cast fused)
void wgrad(const void* dy, const void* x, float* dw_part, float* db_part, long part_stride, long R, int N, int K,
           int H, int W, int Cin, int S, hipStream_t st, bool out_bf16 = false);
// the same for nb <= kWgMaxBatch independent problems of one shape in one launch (grid.y = problem)
constexpr int kWgMaxBatch = 32;
struct WgBatch {
  const void* dy[kWgMaxBatch];
  const void* x[kWgMaxBatch];
  float* dw[kWgMaxBatch];
  float* db[kWgMaxBatch];
};
void wgrad_batched(const WgBatch& P, int nb, long part_stride, long R, int N, int K, int H, int W, int Cin, int S,
                   hipStream_t st, bool out_bf16 = false);

// ---- bo_encoder.hip ----------------------------------------------------------------------------
// fused beginning-build-order transformer (20 tokens, 3 pre-LN layers); weights bf16 or fp32 (wdt),
// LayerNorm affines fp32; bo / loc indices int16 / int32 / int64 (idt 0 / 1 / 2)
constexpr int kBoTokens = 20, kBoLayers = 3, kBoRecord = 11120, kBoGradSize = 76880;
struct BoWeights {
  const void* w0;
  const void* b0;
  const float* ln1w[kBoLayers];
  const float* ln1b[kBoLayers];
  const void* wqkv[kBoLayers];
  const void* bqkv[kBoLayers];
  const void* wp[kBoLayers];
  const void* bp[kBoLayers];
  const float* ln2w[kBoLayers];
  const float* ln2b[kBoLayers];
  const void* w1[kBoLayers];
  const void* b1[kBoLayers];
  const void* w2[kBoLayers];
  const void* b2[kBoLayers];
};
// out [B, 64] fp32 = mean over tokens of the transformer output; save [B, 3, kBoRecord] (nullable)
void bo_encoder_fwd(const void* bo, const void* loc, int idt, const BoWeights& w, int wdt, float* out, float* save,
                    long B, hipStream_t st);
// grad [replicas, kBoGradSize] fp32 (zeroed by the caller; observation b adds into replica b % replicas)
// += parameter gradients for dmean [B, 64]; the caller sums the replicas
void bo_encoder_bwd(const void* bo, const void* loc, int idt, const BoWeights& w, int wdt, const float* save,
                    const float* dmean, float* grad, long B, int replicas, hipStream_t st);

// ---- gemm_k32.hip ------------------------------------------------------------------------------
// out [R][N] = a [R][32] . W [32][N], bf16; wT = W^T [N][32] contiguous; N % 16 == 0
void mm_k32(const void* a, const void* wT, void* out, long R, int N, hipStream_t s);

// ---- resmlp.hip -------------------------------------------------------------------------------
// n <= kResMax x ResFCBlock2(256): x <- LN(fc2(relu(fc1(x))) + x); linear weights / biases bf16, LN fp32
constexpr int kResMax = 16;
struct ResMlpW {
  const void* w1[kResMax];
  const void* b1[kResMax];
  const void* w2[kResMax];
  const void* b2[kResMax];
  const float* g[kResMax];
  const float* be[kResMax];
  const void* pk;             // fragment-ordered GEMM operands [2 n][65536] (resmlp_pack)
};
// out [R, 256] fp32; saved (nullable sv_x): sv_x / sv_h bf16 [n, R, 256], sv_xhat fp32 [n, R, 256], sv_rstd [n, R]
void resmlp_fwd(const void* x0, int x0_dt, const ResMlpW& w, int nblk, float* out, uint16_t* sv_x, uint16_t* sv_h,
                float* sv_xhat, float* sv_rstd, long R, hipStream_t s);
// dst [2 n][65536]: the GEMM operands in the kernels' per-wave fragment order (one 1-KB contiguous
// run per wave load instruction): forward W1_0, W2_0, W1_1, ...; backward (bwd) W2_0^T, W1_0^T, W2_1^T, ...
void resmlp_pack(const ResMlpW& w, int nblk, bool bwd, uint16_t* dst, hipStream_t s);
int resmlp_row_blocks(long R);
// dx0 [R, 256] fp32; sv_dy / sv_dh bf16 [n, R, 256] (for the batched weight gradient);
// ln_part [row_blocks, n, 512] fp32 per-workgroup (dgamma | dbeta) partials
void resmlp_bwd(const float* dout, const ResMlpW& w, int nblk, const uint16_t* sv_h, const float* sv_xhat,
                const float* sv_rstd, uint16_t* sv_dy, uint16_t* sv_dh, float* ln_part, float* dx0, long R,
                hipStream_t s);

// ---- loss.hip ----------------------------------------------------------------------------------
// per row of logits l [R, C] (+ teacher t [R, C], may be null) and action a [R]:
// out [3, R] = (logp_a, entropy, KL(t || l)); stats [R, 6] saved for the backward
void head_stats_fwd(const void* l, int l_dt, const void* t, int t_dt, const long* act, float* out, float* stats, long R,
                    int C, hipStream_t s);
// dl [R, C] (l's dtype) = g_a d(logp_a) + g_H dH + g_KL dKL, g [3, R]
void head_stats_bwd(const void* l, int l_dt, const void* t, int t_dt, const long* act, const float* stats,
                    const float* g, void* dl, long R, int C, hipStream_t s);
// ---- rl_loss.hip: the RL loss after the per-head statistics, with its closed-form gradients (one workgroup)
int rl_loss_info_size(int F);
int rl_loss_max_tb();
void rl_loss(const float* alp, const float* blp, const float* hm, const float* ent, const float* kl, const float* v,
             const float* r, const float* wm, const float* atflag, const float* sc, int F, int T, int B, int upgo_f,
             int only_value, float* dalp, float* dent, float* dkl, float* dv, float* info, hipStream_t s);

// ---- gate_chain.hip: four chained 128 x 128 pointwise layers, activation tile resident in LDS
// layer L: out[L] = epilogue(in @ m[L]^T) with m[L] [128 out][128 in] bf16; epilogue: + bias[L] (fp32,
// nullable), ReLU if bit L of relu_mask, zero where mask[L] (bf16 [P,128], nullable) <= 0, + res[L] (nullable)
struct GateChainArgs {
  const uint16_t* x;
  const uint16_t* m[4];
  const float* bias[4];
  const uint16_t* mask[4];
  const uint16_t* res[4];
  uint16_t* out[4];
  int relu_mask;
};
void gate_chain(const GateChainArgs& a, long P, hipStream_t s);
// the fp32 chain (bf16x6 split products): out[L] = epilogue_L(in_L . m[L]^T), in_0 = x, in_{L+1} = out[L]; the
// epilogue adds bias[L], applies ReLU (relu_mask bit L), zeroes where mask[L] <= 0, adds res[L] (each optional)
struct GateChainF32Args {
  const float* x;
  const float* m[4];
  const float* bias[4];
  const float* mask[4];
  const float* res[4];
  float* out[4];
  int relu_mask;
};
void gate_chain_f32(const GateChainF32Args& a, long P, hipStream_t s);

}  // namespace as
