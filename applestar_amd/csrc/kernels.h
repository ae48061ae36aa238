// Host-side launch entry points of the applestar_amd HIP kernels (gfx950).
// Every launcher takes raw device pointers + an explicit hipStream_t so it can be captured into a
// hipGraph; none allocates or synchronises.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace as {

// dtype codes shared with the bindings
enum DType : int { DT_F32 = 0, DT_BF16 = 1 };

// ---- layernorm.hip -------------------------------------------------------------------------
// y = act(LN(x + residual) * w + b); saves per-row mean/rstd and (if residual) the fp32 sum.
void layer_norm_fwd(const void* x, int x_dt, const void* res, int res_dt, const float* w, const float* b,
                    void* y, int y_dt, float* xsum, float* mean, float* rstd, long rows, int cols, float eps,
                    int act, hipStream_t s);
// dx (fp32 or bf16) and per-block partial dw/db [nblk, cols] (reduced by layer_norm_bwd_reduce).
void layer_norm_bwd(const void* dy, int dy_dt, const void* xin, int xin_dt, const void* y, int y_dt,
                    const float* w, const float* mean, const float* rstd, void* dx, int dx_dt,
                    float* dw_part, float* db_part, long rows, int cols, int act, int nblk, hipStream_t s);
void column_reduce(const float* part, float* out, int nrows, int cols, hipStream_t s);
int layer_norm_bwd_blocks(long rows);

// ---- scan.hip --------------------------------------------------------------------------------
// y[t] = a[t] * y[t+1] + b[t], t = T-1..0, y[T] = init; tensors [K, T, B] fp32 (K independent).
void reverse_scan(const float* a, const float* b, const float* init, float* y, int K, int T, int B,
                  hipStream_t s);

// ---- elementwise.hip -------------------------------------------------------------------------
// out = relu(tanh(y * sigmoid(g)) * sp + x)
void gated_residual_fwd(const void* y, const void* g, const float* sp, const void* x, void* out, int dt, long n,
                        hipStream_t s);
void gated_residual_bwd(const void* dout, const void* y, const void* g, const float* sp, const void* out, int dt,
                        void* dy, void* dg, void* dx, float* dsp_part, long n, int nblk, hipStream_t s);
int elementwise_blocks(long n);

// ---- lstm.hip --------------------------------------------------------------------------------
// LayerNorm-LSTM recurrence for H in {384, 32}. xp [T,B,4H] = LN_i(x W_ih^T); wT = W_hh^T [H][4H]
// (fp32 or bf16). Saves what BPTT needs: c_all [T+1,B,H], xhat_h/gates [T,B,4H], xhat_c [T,B,H],
// rstd_h/rstd_c [T,B].
bool lnlstm_supported(int H);
void lnlstm_fwd(const float* xp, const float* h0, const float* c0, const void* wT, int w_dt, const float* lnh_w,
                const float* lnh_b, const float* lnc_w, const float* lnc_b, int T, int B, int H, float eps, float* out,
                float* c_all, float* xhat_h, float* rstd_h, float* gates, float* xhat_c, float* rstd_c, float* hT,
                float* cT, hipStream_t s);
// w = W_hh [4H][H]. Outputs d(xp) [T,B,4H], d(h W_hh^T) [T,B,4H], dL/d(LN_c out) [T,B,H], dh0, dc0.
void lnlstm_bwd(const float* dout, const float* dhT, const float* dcT, const float* gates, const float* c_all,
                const float* xhat_c, const float* rstd_c, const float* xhat_h, const float* rstd_h, const void* w,
                int w_dt, const float* lnh_w, const float* lnc_w, int T, int B, int H, float* dgates, float* dhg,
                float* dc_ln, float* dh0, float* dc0, hipStream_t s);

}  // namespace as
