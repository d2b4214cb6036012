// nrc_train_dc.hip — the Frequency training step's forward / loss / backward / per-block dW kernel, "decoupled
// chain" form (round 3). Reference: Network::train -> trainer->training_step (nrc/src/NRCNetwork.cu:41-56), tcnn
// FullyFusedMLP forward + backward with RelativeL2Luminance; numerics and slab format
// are those of train16_split_kernel (nrc_train16.hip), which it replaces.
//
// Why a new form. The round-2 kernel staged both weight images (82 KiB) into LDS per block and moved every wave of the
// block through one barrier per forward layer and one per backward step; a block was a ~16k-cycle latency chain at
// 128 samples and the grid had one block per 128 samples, so a 2,048-sample minibatch (configs[3]: 16,384 split over
// 8 ranks) ran 16 blocks on a 256-CU chip. Here:
//   * a block is CW "chain" waves x GPW groups x 16 samples (S = 16..128 samples; 16 at 2,048 samples -> 128 blocks)
//     plus DWW "dW" waves;
//   * a chain wave streams its A fragments straight from the L2-resident f16 images into registers, two layers ahead
//     of their use (no LDS staging, no wait on other waves' DMAs, no barrier in the forward pass);
//   * it writes every activation image ([sample][feature], the t16 swizzle) once, in the forward pass, and each
//     delta image in the backward pass, then bumps an LDS counter (ready[L]); the dW waves poll that counter,
//     compute dW_L = delta_L in_L^T over the block's S samples from transposed LDS reads and stream the f16 tiles to
//     the block's slab. The only wait of the chain on the dW waves is the reuse of a delta buffer (a ring of two),
//     i.e. when the dW waves fall two steps behind.
// The MFMA sequences per accumulator are train16_split_kernel's, so at S = 128 the slabs are bitwise the same.
#include "nrc_t16.h"

namespace nrc_amd {
namespace {
using namespace t16;

template <int CW, int GPW>
struct DcLayout {
    static constexpr int S = 16 * GPW * CW;  // samples per block
    static constexpr int IMG = 128 * S;      // one [S][64] f16 image (128-B rows)
    static constexpr int OFF_A = 0;          // a_0 .. a_4 (outputs of layers 0..4 = inputs of layers 1..5)
    static constexpr int OFF_X0 = 5 * IMG;   // layer-0 K slots 0..63
    static constexpr int OFF_D5 = 6 * IMG;   // delta_5 (quads 0..3)
    static constexpr int OFF_D = 7 * IMG;    // delta_4 .. delta_0, ring of two buffers
    static constexpr int OFF_X2 = 9 * IMG;   // layer-0 K slots 64..95 ([S][32], 64-B rows)
    static constexpr int OFF_FLAGS = OFF_X2 + 64 * S;
    static constexpr int BYTES = OFF_FLAGS + 64;
};
static_assert(DcLayout<4, 2>::BYTES <= 160 * 1024, "LDS budget at 128 samples per block");

// flags: ready[0..5] (chain waves that published delta_L), red[0..3] (loss partials), dwdone[L] (dW waves that finished
// their step L, for the steps L = 2..4 whose delta buffer the chain reuses).
// Round 3 fix: one counter of ALL dW-wave steps let a dW wave that ran ahead into step L - 1 stand in for a slow one still
// reading delta_L, and the chain overwrote that buffer under it (nondeterministic dW_2..dW_4 in 5 of 6 trials once a
// slower loss-partial store delayed dW wave 0); the chain now waits for every dW wave's step L + 1 exactly.
constexpr int kFlagRed = 8;
constexpr int flag_dwdone(int L) { return 12 + (L - 2); }  // L = 2, 3, 4 -> 12, 13, 14

__device__ __forceinline__ uint32_t lds_load(const uint32_t* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
// bounded (2^20 polls, tens of ms) so that a protocol error cannot hang the GPU; a wave that gives up sets the launch's
// error word (host-mapped, nrc_net::proto_err), which the host turns into NRC_ERR_INTERNAL at its next check (round 4:
// before, a timeout gave a wrong gradient with NRC_OK)
constexpr int kPollBound = 1 << 20;
__device__ __forceinline__ void lds_wait_ge(const uint32_t* p, uint32_t v, uint32_t* err, int lane) {
    int i = 0;
    for (; lds_load(p) < v && i < kPollBound; ++i) __builtin_amdgcn_s_sleep(1);
    if (i == kPollBound && lane == 0) __hip_atomic_store(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    asm volatile("" ::: "memory");  // no LDS read of the published data above the poll
}
// publish: this wave's LDS writes have landed (lgkmcnt), then one lane bumps the counter
__device__ __forceinline__ void lds_publish(uint32_t* p, int lane) {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if (lane == 0) __hip_atomic_fetch_add(p, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

__device__ __forceinline__ void load8(const h8* __restrict__ img, int layer_frag0, int lane, h8 (&w)[8]) {
#pragma unroll
    for (int i = 0; i < 8; ++i) w[i] = img[(layer_frag0 + i) * 64 + lane];
}

// ---- chain wave: encode, forward, loss, delta chain; publishes images for the dW waves
// STAMP (diagnostic build, nrc_debug_train_stamps): s_memtime at phase boundaries, lane 0 -> stamps[wave][16]
template <bool STAMP>
struct Stamper {
    uint64_t* p;
    int lane;
    __device__ __forceinline__ void operator()(int k) const {
        if constexpr (STAMP) {
            __builtin_amdgcn_sched_barrier(0);
            const uint64_t t = __builtin_amdgcn_s_memtime();
            __builtin_amdgcn_sched_barrier(0);
            if (lane == 0) p[k] = t;
        }
    }
    __device__ __forceinline__ void real(int k) const {
        if constexpr (STAMP) {
            __builtin_amdgcn_sched_barrier(0);
            const uint64_t t = __builtin_amdgcn_s_memrealtime();
            __builtin_amdgcn_sched_barrier(0);
            if (lane == 0) p[k] = t;
        }
    }
};

template <int CW, int GPW, int DWW, bool STAMP, bool PADQ = false>  // PADQ: padded RadianceQuery records
__device__ __forceinline__ void dc_chain(const float* __restrict__ q, const float* __restrict__ t, int64_t b,
                                         float n_total, float loss_scale, const h8* __restrict__ wf,
                                         const h8* __restrict__ wb, char* smem, int cw, int lane, uint32_t* err,
                                         const Stamper<STAMP>& stamp) {
    using Lay = DcLayout<CW, GPW>;
    constexpr int S = Lay::S;
    uint32_t* flags = (uint32_t*)(smem + Lay::OFF_FLAGS);
    char* const img_x0 = smem + Lay::OFF_X0;
    char* const img_x2 = smem + Lay::OFF_X2;
    char* const img_d5 = smem + Lay::OFF_D5;
    const int g = lane >> 4, c = lane & 15;
    const int gg = g < 3 ? g : 0;

    // sample loads first, then the first three layers' fragments (layer l + 2 is loaded while layer l computes)
    int r[GPW];
    bool valid[GPW];
    float pq[GPW][3], bl[GPW][2], iv[GPW][2], tg[GPW][3];
    [[maybe_unused]] float pad[GPW];
    constexpr int X = PADQ ? 1 : 0;
#pragma unroll
    for (int u = 0; u < GPW; ++u) {
        r[u] = 16 * GPW * cw + 16 * u + c;
        const int64_t s = (int64_t)blockIdx.x * S + r[u];
        valid[u] = s < b;
        const int64_t sc = valid[u] ? s : b - 1;
        // position (+ pad_), OneBlob dims 3 + 2g, 4 + 2g, Identity dims 9 + 2g, 10 + 2g (lane group 3: dummies with
        // zero weights, fed from group 0's dims so that they stay finite), target
        const float* qr = q + sc * (NRC_INPUT_DIMS + X);
#pragma unroll
        for (int k = 0; k < 3; ++k) pq[u][k] = qr[k];
        if constexpr (PADQ) pad[u] = qr[3];
        bl[u][0] = qr[3 + X + 2 * gg];
        bl[u][1] = qr[4 + X + 2 * gg];
        iv[u][0] = qr[9 + X + 2 * gg];
        iv[u][1] = qr[10 + X + 2 * gg];
#pragma unroll
        for (int k = 0; k < 3; ++k) tg[u][k] = t[sc * 3 + k];
    }
    h8 w0[12], wA[8], wB[8], wC[8];
#pragma unroll
    for (int mb = 0; mb < 4; ++mb)
#pragma unroll
        for (int ks = 0; ks < 3; ++ks) w0[mb * 3 + ks] = wf[t16_fwd_frag(0, mb, ks) * 64 + lane];
    load8(wf, t16_fwd_frag(1, 0, 0), lane, wA);
    load8(wf, t16_fwd_frag(2, 0, 0), lane, wB);
    __builtin_amdgcn_sched_barrier(0);

    // encode; K slots 0..63 / 64..95 to their images (read by the last dW step)
    h8 x[GPW][3];
#pragma unroll
    for (int u = 0; u < GPW; ++u) {
        if constexpr (PADQ) encode16(pq[u][0], pq[u][1], pq[u][2], bl[u][0], bl[u][1], iv[u][0], iv[u][1], g, x[u], pad[u]);
        else encode16(pq[u][0], pq[u][1], pq[u][2], bl[u][0], bl[u][1], iv[u][0], iv[u][1], g, x[u]);
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
            const u4 w = __builtin_bit_cast(u4, x[u][ks]);
            *(u2*)(img_x0 + off64(r[u], 8 * ks + 2 * g)) = u2{w.x, w.y};
            *(u2*)(img_x0 + off64(r[u], 8 * ks + 2 * g + 1)) = u2{w.z, w.w};
        }
        const u4 w = __builtin_bit_cast(u4, x[u][2]);
        *(u2*)(img_x2 + off32(r[u], 2 * g)) = u2{w.x, w.y};
        *(u2*)(img_x2 + off32(r[u], 2 * g + 1)) = u2{w.z, w.w};
    }
    int wo[GPW][4];
#pragma unroll
    for (int u = 0; u < GPW; ++u) row_offsets(r[u], g, wo[u]);
    stamp(1);

    // ---- forward
    h8 a[5][GPW][2];
    f4 cc[GPW][4];
#pragma unroll
    for (int mb = 0; mb < 4; ++mb)
#pragma unroll
        for (int u = 0; u < GPW; ++u) {
            cc[u][mb] = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int ks = 0; ks < 3; ++ks) cc[u][mb] = mfma16(w0[mb * 3 + ks], x[u][ks], cc[u][mb]);
        }
#pragma unroll
    for (int u = 0; u < GPW; ++u) {
        a[0][u][0] = relu_b(cc[u][0], cc[u][1]);
        a[0][u][1] = relu_b(cc[u][2], cc[u][3]);
        put_rows64(smem + Lay::OFF_A, wo[u], a[0][u]);
    }
    load8(wf, t16_fwd_frag(3, 0, 0), lane, wC);
    __builtin_amdgcn_sched_barrier(0);
    stamp(2);

    auto hidden = [&](const h8 (&w)[8], int l) {  // layer l = 1..4: a[l] from a[l - 1]
#pragma unroll
        for (int mb = 0; mb < 4; ++mb)
#pragma unroll
            for (int u = 0; u < GPW; ++u) {
                cc[u][mb] = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
                for (int ks = 0; ks < 2; ++ks) cc[u][mb] = mfma16(w[mb * 2 + ks], a[l - 1][u][ks], cc[u][mb]);
            }
#pragma unroll
        for (int u = 0; u < GPW; ++u) {
            a[l][u][0] = relu_b(cc[u][0], cc[u][1]);
            a[l][u][1] = relu_b(cc[u][2], cc[u][3]);
            put_rows64(smem + Lay::OFF_A + l * Lay::IMG, wo[u], a[l][u]);
        }
    };
    hidden(wA, 1);
    load8(wf, t16_fwd_frag(4, 0, 0), lane, wA);
    __builtin_amdgcn_sched_barrier(0);
    stamp(3);
    hidden(wB, 2);
    h8 w5[2];
    h4 w5t[4];
    w5[0] = wf[t16_fwd_frag(5, 0, 0) * 64 + lane];
    w5[1] = wf[t16_fwd_frag(5, 0, 1) * 64 + lane];
    {
        const h4* wb4 = (const h4*)wb;
#pragma unroll
        for (int mb = 0; mb < 4; ++mb) w5t[mb] = wb4[t16_bwd_frag(5, mb, 0) * 128 + lane];
    }
    __builtin_amdgcn_sched_barrier(0);
    stamp(4);
    hidden(wC, 3);
    load8(wb, t16_bwd_frag(4, 0, 0), lane, wC);
    __builtin_amdgcn_sched_barrier(0);
    stamp(5);
    hidden(wA, 4);
    load8(wb, t16_bwd_frag(3, 0, 0), lane, wA);
    __builtin_amdgcn_sched_barrier(0);
    stamp(6);
    f4 o[GPW];
#pragma unroll
    for (int u = 0; u < GPW; ++u) {
        o[u] = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) o[u] = mfma16(w5[ks], a[4][u][ks], o[u]);
    }
    load8(wb, t16_bwd_frag(2, 0, 0), lane, wB);
    __builtin_amdgcn_sched_barrier(0);
    stamp(7);

    // ---- loss, delta_5 (published with the loss partial)
    float lossv = 0.0f;
    h4 d5[GPW];
#pragma unroll
    for (int u = 0; u < GPW; ++u) d5[u] = loss_delta5(o[u], tg[u], valid[u], g, n_total, loss_scale, lossv);
    lossv = row_sum16(lossv);  // lane group 0 = row 0 holds every nonzero term
    if (lane == 0) ((float*)(flags + kFlagRed))[cw] = lossv;
#pragma unroll
    for (int u = 0; u < GPW; ++u) *(h4*)(img_d5 + off64(r[u], g)) = d5[u];
    lds_publish(flags + 5, lane);
    stamp(8);

    // ---- backward. step 5: delta_4 = W5^T delta_5 * [a_4 > 0] (16x16x16: K = the 16 output rows) -> buffer 0
    h8 d[GPW][2], dn[GPW][2];
#pragma unroll
    for (int u = 0; u < GPW; ++u) {
        f4 c5[4];
#pragma unroll
        for (int mb = 0; mb < 4; ++mb) c5[mb] = mfma16k16(w5t[mb], d5[u], f4{0.f, 0.f, 0.f, 0.f});
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) d[u][s2] = gate_b(c5[2 * s2], c5[2 * s2 + 1], a[4][u][s2]);
        put_rows64(smem + Lay::OFF_D, wo[u], d[u]);
    }
    lds_publish(flags + 4, lane);
    __builtin_amdgcn_sched_barrier(0);
    stamp(9);

    // steps L = 4..1: delta_{L-1} = (W_L^T delta_L) * [a_{L-1} > 0] into buffer (L - 1) & 1; from L = 3 on the buffer's
    // previous delta (delta_{L+1}) must have been read by every dW wave (their step L + 1)
    auto step = [&](const h8 (&w)[8], int L) {
        h8 W[4][2];
#pragma unroll
        for (int mb = 0; mb < 4; ++mb) {
            W[mb][0] = w[2 * mb];
            W[mb][1] = w[2 * mb + 1];
        }
        chain_groups<GPW>(W, d, a[L - 1], dn);
        if (L <= 3) lds_wait_ge(flags + flag_dwdone(L + 1), (uint32_t)DWW, err, lane);  // buffer (L-1)&1 held delta_{L+1}
        char* const buf = smem + Lay::OFF_D + ((L - 1) & 1) * Lay::IMG;
#pragma unroll
        for (int u = 0; u < GPW; ++u) {
            put_rows64(buf, wo[u], dn[u]);
#pragma unroll
            for (int s2 = 0; s2 < 2; ++s2) d[u][s2] = dn[u][s2];
        }
        lds_publish(flags + (L - 1), lane);
    };
    step(wC, 4);
    load8(wb, t16_bwd_frag(1, 0, 0), lane, wC);
    __builtin_amdgcn_sched_barrier(0);
    stamp(10);
    step(wA, 3);
    __builtin_amdgcn_sched_barrier(0);
    stamp(11);
    step(wB, 2);
    __builtin_amdgcn_sched_barrier(0);
    stamp(12);
    step(wC, 1);
    stamp(13);
}

// Transposed-read operand of one 16-feature tile of a [S][*] image over the block's samples: k-step kk covers
// samples 32 kk .. 32 kk + 31 (S >= 32, two ds_read_b64_tr_b16 per lane: rows 8G + q and 8G + 4 + q) or, at S = 16,
// the 16 samples as a 16x16x16 operand (one read: rows 4G + q).
template <int S>
struct DwOps {
    static constexpr int KK = S >= 32 ? S / 32 : 1;
    h8 v[KK];
};

template <int S, int ROWB>
__device__ __forceinline__ void dw_load(const char* img, int quad, int lane, DwOps<S>& op) {
    const int G = lane >> 4, qq = (lane >> 2) & 3, pp = lane & 3;
    auto off = [&](int rr) { return ROWB == 128 ? off64(rr, quad + pp) : off32(rr, quad + pp); };
    if constexpr (S >= 32) {
        const int r0 = 8 * G + qq;
#pragma unroll
        for (int kk = 0; kk < S / 32; ++kk)
            op.v[kk] = tr_pair(img + off(r0) + kk * 32 * ROWB, img + off(r0 + 4) + kk * 32 * ROWB);
    } else {
        const h4 x = tr16(img + off(4 * G + qq));
        op.v[0] = __builtin_shufflevector(x, x, 0, 1, 2, 3, 0, 1, 2, 3);
    }
}

template <int S>
__device__ __forceinline__ f4 dw_mfma(const DwOps<S>& A, const DwOps<S>& B) {
    f4 acc = {0.f, 0.f, 0.f, 0.f};
    if constexpr (S >= 32) {
#pragma unroll
        for (int kk = 0; kk < S / 32; ++kk) acc = mfma16(A.v[kk], B.v[kk], acc);
    } else {
        acc = mfma16k16(__builtin_shufflevector(A.v[0], A.v[0], 0, 1, 2, 3),
                        __builtin_shufflevector(B.v[0], B.v[0], 0, 1, 2, 3), acc);
    }
    return acc;
}

// ---- dW wave: dW_L tile pairs (tm, 2p), (tm, 2p + 1) of this wave, L = 5..0. Per step every operand read of the
// wave's pairs is issued before the first MFMA (one LDS round trip per step instead of one per pair); a wave past the
// step's last pair (L = 5 at DWW = 4) recomputes that pair and does not store it.
template <int L>
constexpr int dc_npairs() { return L == 5 ? 2 : L == 0 ? 12 : 8; }

template <int CW, int GPW, int DWW, int L, bool STAMP>
__device__ __forceinline__ void dc_dw_step(char* smem, int dw, int lane, _Float16* __restrict__ slab,
                                           float* __restrict__ loss_partials, uint32_t* err,
                                           const Stamper<STAMP>& stamp) {
    using Lay = DcLayout<CW, GPW>;
    constexpr int S = Lay::S;
    constexpr int NP = dc_npairs<L>();
    constexpr int PER = (NP + DWW - 1) / DWW;
    uint32_t* flags = (uint32_t*)(smem + Lay::OFF_FLAGS);
    lds_wait_ge(flags + L, (uint32_t)CW, err, lane);
    stamp(1 + 2 * (5 - L));
    if (L == 5 && dw == 0 && lane == 0) {
        const float* red = (const float*)(flags + kFlagRed);
        float lp;
        if constexpr (CW == 4) lp = (red[0] + red[1]) + (red[2] + red[3]);
        else if constexpr (CW == 2) lp = red[0] + red[1];
        else lp = red[0];
        loss_partials[blockIdx.x] = lp;
    }
    const char* imgd = L == 5 ? smem + Lay::OFF_D5 : smem + Lay::OFF_D + (L & 1) * Lay::IMG;
    const char* imgi = L >= 1 ? smem + Lay::OFF_A + (L - 1) * Lay::IMG : smem + Lay::OFF_X0;
    int tm[PER], tp[PER];
    bool own[PER];
    DwOps<S> A[PER], Be[PER], Bo[PER];
#pragma unroll
    for (int k = 0; k < PER; ++k) {
        const int i0 = dw + k * DWW;
        own[k] = i0 < NP;
        const int i = own[k] ? i0 : NP - 1;
        tm[k] = L == 0 ? i / 3 : L == 5 ? 0 : i >> 1;
        tp[k] = L == 0 ? i % 3 : L == 5 ? i : i & 1;
        dw_load<S, 128>(imgd, 4 * tm[k], lane, A[k]);
        if (L == 0 && tp[k] == 2) {
            dw_load<S, 64>(smem + Lay::OFF_X2, 0, lane, Be[k]);
            dw_load<S, 64>(smem + Lay::OFF_X2, 4, lane, Bo[k]);
        } else {
            dw_load<S, 128>(imgi, 8 * tp[k], lane, Be[k]);
            dw_load<S, 128>(imgi, 8 * tp[k] + 4, lane, Bo[k]);
        }
    }
    f4 acc[PER][2];
#pragma unroll
    for (int k = 0; k < PER; ++k) {
        acc[k][0] = dw_mfma<S>(A[k], Be[k]);
        acc[k][1] = dw_mfma<S>(A[k], Bo[k]);
    }
    // every read of delta_L by this wave has returned (the MFMAs consumed them): release the buffer, then store
    if (L >= 2 && L <= 4) lds_publish(flags + flag_dwdone(L), lane);
#pragma unroll
    for (int k = 0; k < PER; ++k)
        if (own[k]) slab_pair_b<16>(slab, L, tm[k], 2 * tp[k], lane, pack_pair(acc[k][0], acc[k][1]));
    stamp(2 + 2 * (5 - L));
}

#if NRC_DEBUG_KERNELS
// debug knob dc_dw0_delay: dW wave 0 idles this many s_sleep(127) rounds after its step 5, so that the other dW waves run
// ahead of it (the stress case of the round-3 ring-buffer race, tests/test_gpu_train_dc.py)
__device__ int g_dc_dw0_delay = 0;
#endif

template <int CW, int GPW, int DWW, bool STAMP>
__device__ __forceinline__ void dc_dw(char* smem, int dw, int lane, _Float16* __restrict__ slab,
                                      float* __restrict__ loss_partials, uint32_t* err, const Stamper<STAMP>& stamp) {
    dc_dw_step<CW, GPW, DWW, 5, STAMP>(smem, dw, lane, slab, loss_partials, err, stamp);
#if NRC_DEBUG_KERNELS
    if (dw == 0)
        for (int i = 0; i < g_dc_dw0_delay; ++i) __builtin_amdgcn_s_sleep(127);
#endif
    dc_dw_step<CW, GPW, DWW, 4, STAMP>(smem, dw, lane, slab, loss_partials, err, stamp);
    dc_dw_step<CW, GPW, DWW, 3, STAMP>(smem, dw, lane, slab, loss_partials, err, stamp);
    dc_dw_step<CW, GPW, DWW, 2, STAMP>(smem, dw, lane, slab, loss_partials, err, stamp);
    dc_dw_step<CW, GPW, DWW, 1, STAMP>(smem, dw, lane, slab, loss_partials, err, stamp);
    dc_dw_step<CW, GPW, DWW, 0, STAMP>(smem, dw, lane, slab, loss_partials, err, stamp);
}

template <int CW, int GPW, int DWW, bool STAMP = false, bool PADQ = false>
__global__ __launch_bounds__(64 * (CW + DWW), (CW + DWW + 3) / 4) void train_dc_kernel(
    const float* __restrict__ q, const float* __restrict__ t, int64_t b, float n_total, float loss_scale,
    const h8* __restrict__ wf, const h8* __restrict__ wb, _Float16* __restrict__ slabs, float* __restrict__ loss_partials,
    uint32_t* err, uint64_t* __restrict__ stamps) {
    using Lay = DcLayout<CW, GPW>;
    __shared__ __attribute__((aligned(16))) char smem[Lay::BYTES];
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const Stamper<STAMP> stamp{STAMP ? stamps + ((int64_t)blockIdx.x * (CW + DWW) + wave) * 16 : nullptr, lane};
    stamp.real(14);
    stamp(0);
    if (threadIdx.x < 16) ((uint32_t*)(smem + Lay::OFF_FLAGS))[threadIdx.x] = 0;
    __syncthreads();
    if (wave < CW)
        dc_chain<CW, GPW, DWW, STAMP, PADQ>(q, t, b, n_total, loss_scale, wf, wb, smem, wave, lane, err, stamp);
    else
        dc_dw<CW, GPW, DWW, STAMP>(smem, wave - CW, lane, slabs + (int64_t)blockIdx.x * slab_floats(0), loss_partials,
                                   err, stamp);
    stamp.real(15);
}

template <int CW, int GPW, int DWW, bool PADQ = false>
hipError_t launch_dc(const float* q, const float* t, int64_t b, float n_total, float loss_scale, const _Float16* wf,
                     const _Float16* wb, _Float16* slabs, float* loss_partials, uint32_t* err, hipStream_t s,
                     uint64_t* stamps) {
    constexpr int S = DcLayout<CW, GPW>::S;
    const int blocks = (int)((b + S - 1) / S);
    if constexpr (PADQ) {  // padded RadianceQuery records: no stamped build
        if (stamps) return hipErrorNotSupported;
        hipLaunchKernelGGL((train_dc_kernel<CW, GPW, DWW, false, true>), dim3(blocks), dim3(64 * (CW + DWW)), 0, s, q,
                           t, b, n_total, loss_scale, (const h8*)wf, (const h8*)wb, slabs, loss_partials, err, nullptr);
        return hipGetLastError();
    }
#if NRC_DEBUG_KERNELS
    if (stamps)
        hipLaunchKernelGGL((train_dc_kernel<CW, GPW, DWW, true>), dim3(blocks), dim3(64 * (CW + DWW)), 0, s, q, t, b,
                           n_total, loss_scale, (const h8*)wf, (const h8*)wb, slabs, loss_partials, err, stamps);
    else
#else
    if (stamps) return hipErrorNotSupported;  // stamped builds live in libnrc_amd_debug.so
#endif
        hipLaunchKernelGGL((train_dc_kernel<CW, GPW, DWW>), dim3(blocks), dim3(64 * (CW + DWW)), 0, s, q, t, b,
                           n_total, loss_scale, (const h8*)wf, (const h8*)wb, slabs, loss_partials, err, nullptr);
    return hipGetLastError();
}

}  // namespace

// Shapes (samples per block S = 16 GPW CW): selected by dc_shape(b) unless a caller forces one.
int dc_samples_per_block(int shape) {
    switch (shape) {
        case 0: return 16;   // CW 1, GPW 1, DWW 1
        case 1: return 32;   // CW 1, GPW 2, DWW 1
        case 2: return 64;   // CW 2, GPW 2, DWW 2
        case 3: return 128;  // CW 4, GPW 2, DWW 4 (slabs bitwise those of train16_split_kernel)
        case 4: return 64;   // CW 4, GPW 1, DWW 4
        case 5: return 32;   // CW 2, GPW 1, DWW 2
        case 6: return 16;   // CW 1, GPW 1, DWW 2
        case 7: return 32;   // CW 2, GPW 1, DWW 4
        default: return 0;
    }
}

// Production shape by batch size (in-process A/B, tools/ab_train_dc.py, profiles/r03_train/): a data-parallel rank's
// slice (b <= 4,096) in 32-sample blocks of 2 chain + 4 dW waves, so that it spreads over the chip (2,048 samples: 64
// blocks; step 10.3 vs 11.4 us for round 2's kernel in 128-sample blocks); -1 = the full minibatch stays on round 2's
// role-split kernel (nrc_train16.hip; 12.7 us at 16,384 against 13.7 for the same 128-sample blocks here -- at that
// size every CU holds a block and the LDS-staged weight images beat per-wave register streams).
int dc_auto_shape(int64_t b) { return b <= 4096 ? 7 : -1; }

int dc_waves_per_block(int shape) {
    switch (shape) {
        case 0: case 1: return 2;
        case 2: case 5: return 4;
        case 3: case 4: return 8;
        case 6: return 3;
        case 7: return 6;
        default: return 0;
    }
}

hipError_t launch_train_dc(int shape, const float* queries, const float* targets, int64_t b, float n_total,
                           float loss_scale, const _Float16* wf, const _Float16* wb, _Float16* slabs,
                           float* loss_partials, uint32_t* err, hipStream_t s, uint64_t* stamps, bool padq) {
    if (b <= 0) return hipSuccess;
    if (!err) return hipErrorInvalidValue;
    if (padq) {  // padded RadianceQuery records: the production shape (dc_auto_shape) only
        if (shape != 7) return hipErrorNotSupported;
        return launch_dc<2, 1, 4, true>(queries, targets, b, n_total, loss_scale, wf, wb, slabs, loss_partials, err, s,
                                        stamps);
    }
#if NRC_DEBUG_KERNELS
    static int applied = 0;
    const int delay = std::max(knob(kKnobDcDw0Delay), 0);
    if (delay != applied) {
        const hipError_t e = hipMemcpyToSymbol(HIP_SYMBOL(g_dc_dw0_delay), &delay, sizeof(int));
        if (e != hipSuccess) return e;
        applied = delay;
    }
#endif
    switch (shape) {
        case 0: return launch_dc<1, 1, 1>(queries, targets, b, n_total, loss_scale, wf, wb, slabs, loss_partials, err, s, stamps);
        case 1: return launch_dc<1, 2, 1>(queries, targets, b, n_total, loss_scale, wf, wb, slabs, loss_partials, err, s, stamps);
        case 2: return launch_dc<2, 2, 2>(queries, targets, b, n_total, loss_scale, wf, wb, slabs, loss_partials, err, s, stamps);
        case 3: return launch_dc<4, 2, 4>(queries, targets, b, n_total, loss_scale, wf, wb, slabs, loss_partials, err, s, stamps);
        case 4: return launch_dc<4, 1, 4>(queries, targets, b, n_total, loss_scale, wf, wb, slabs, loss_partials, err, s, stamps);
        case 5: return launch_dc<2, 1, 2>(queries, targets, b, n_total, loss_scale, wf, wb, slabs, loss_partials, err, s, stamps);
        case 6: return launch_dc<1, 1, 2>(queries, targets, b, n_total, loss_scale, wf, wb, slabs, loss_partials, err, s, stamps);
        case 7: return launch_dc<2, 1, 4>(queries, targets, b, n_total, loss_scale, wf, wb, slabs, loss_partials, err, s, stamps);
        default: return hipErrorInvalidValue;
    }
}

}  // namespace nrc_amd
