// nrc_train16.hip — the Frequency training step's forward / loss / backward / per-block dW kernel on
// v_mfma_f32_16x16x32_f16 (round 2). Replaces train_kernel (nrc_kernels.hip, 32x32x16, one 32-sample wave per SIMD)
// for InputEncoding::Frequency; reference: Network::train -> trainer->training_step (nrc/src/NRCNetwork.cu:41-56),
// tcnn FullyFusedMLP forward + backward with RelativeL2Luminance.
//
// One block = 4 waves x 2 groups x 16 samples = 128 samples (so the slab count and the reduction are unchanged), one
// wave per SIMD. Lane l = (g = l >> 4, c = l & 15) works on sample c of each of its wave's two groups; every operand
// stays in the 16x16 C/D layout (lane (g, c) holds rows 4g .. 4g + 3 of column c), which is the next layer's B operand
// with the K order permuted (t16_row) and absorbed into the weight images (nrc_internal.h "t16"). Each weight
// fragment read from LDS feeds both groups' MFMAs: a first version with 8 waves x 16 samples read every fragment
// once per 16 samples and was bound by LDS bandwidth (160 KiB of reads per backward step, 1,850 cycles per step).
//
//   encode (96 K slots, t16_slot_feature) -> forward L0..L5 (46 MFMAs per wave, A fragments from the LDS-DMA'd
//   forward image) -> RelativeL2Luminance on the f16 output, loss-scaled -> per layer L = 5..0, between two
//   barriers: dW_L = delta_L a_{L-1}^T over the block's 128 samples (16x16 tiles from transposed LDS reads of the
//   [sample][feature] images) and delta_{L-1} = (W_L^T delta_L) * [a_{L-1} > 0] (register chain, backward image in
//   LDS), the next layer's images written to the other buffer, the dW tiles streamed to the block's slab.
#include "nrc_t16.h"
#include "nrc_hash.h"

#include <type_traits>

namespace nrc_amd {
namespace {

using namespace t16;

// LDS carve-up (bytes). The four [128][64] f16 images (deltas and activations, double-buffered) sit at offset 0, so
// that an image access is one per-lane offset VGPR plus an immediate (the 16-bit DS offset field reaches every image);
// then the [128][32] image of layer-0 K slots 64..95, the loss partials, the backward image (36 KiB) and the forward
// image (46 KiB + 2 KiB that the fixed-count LDS-DMA overruns into).
constexpr int kImg = 128 * 128;
constexpr int kOffImg = 0;
constexpr int kOffX2 = 4 * kImg;                          // 65536
constexpr int kOffRed = kOffX2 + 128 * 64;                // 73728
constexpr int kOffWb = kOffRed + 256;                     // 73984
constexpr int kOffWf = kOffWb + kT16BwdFrags * 1024;      // 110848
constexpr int kLds = kOffWf + 48 * 1024;                  // 160000
static_assert(kLds <= 160 * 1024, "LDS budget");

// dW tiles into the block's slab as f16 (t16_slab_pos: column pairs, one 16-byte store per lane for both tiles of a
// pair). The slab stores cost the wave a few tens of cycles per store instruction (the CU's stores queue behind one
// another), so the count of store instructions sets their price: f32 tiles, one dwordx4 each, cost ~600 cycles per
// backward step (ablation NRC_T16_ABL=1). f16 pairs halve the instructions; rounding a 128-sample partial to f16 adds
// 2e-5 .. 7e-5 rel-L2 to the summed gradient (oracle partials over 64 training steps) -- tcnn's own
// gradient is f16.
__device__ __forceinline__ void slab_pair(_Float16* __restrict__ slab, int L, int tm, int tn_even, int lane, const u4& v) {
    __builtin_nontemporal_store(v, (u4*)(slab + t16_slab_base(L, tm, tn_even)) + lane);
}
__device__ __forceinline__ void slab_single(_Float16* __restrict__ slab, int L, int tm, int tn, int lane, const f4& v) {
    __builtin_nontemporal_store(u2{pk2(v[0], v[1]), pk2(v[2], v[3])}, (u2*)(slab + t16_slab_pos(L, tm, tn, lane, 0)));
}

// Transposed-read operand of one 16-feature tile over the block's 128 samples (4 k-steps of 32): the lane's byte
// offsets of its two reads (samples 8G + q and 8G + 4 + q of each k-step) and the image's bytes per 32 samples.
struct TrTile {
    const char* img;
    int o0, o1, stride;
};
__device__ __forceinline__ h8 tr_op(const TrTile& t, int kk) {
    return tr_pair(t.img + t.o0 + t.stride * kk, t.img + t.o1 + t.stride * kk);
}

// dW tiles A_i x B_j (i < NA, j < NB) over 128 samples: A = delta-image tiles (rows), B = activation-image tiles
// (columns). Every operand read is issued before the first MFMA.
template <int NA, int NB, int KS = 4>  // KS k-steps of 32 samples (the block's samples)
__device__ __forceinline__ void dw_tiles(const TrTile (&ta)[NA], const TrTile (&tb)[NB], f4 (&acc)[NA][NB]) {
    h8 A[NA][KS], B[NB][KS];
#pragma unroll
    for (int i = 0; i < NA; ++i)
#pragma unroll
        for (int kk = 0; kk < KS; ++kk) A[i][kk] = tr_op(ta[i], kk);
#pragma unroll
    for (int j = 0; j < NB; ++j)
#pragma unroll
        for (int kk = 0; kk < KS; ++kk) B[j][kk] = tr_op(tb[j], kk);
#pragma unroll
    for (int i = 0; i < NA; ++i)
#pragma unroll
        for (int j = 0; j < NB; ++j) acc[i][j] = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kk = 0; kk < KS; ++kk)
#pragma unroll
        for (int i = 0; i < NA; ++i)
#pragma unroll
            for (int j = 0; j < NB; ++j) acc[i][j] = mfma16(A[i][kk], B[j][kk], acc[i][j]);
}

// backward fragments of W_L^T (L = 1..4), 4 M-blocks x 2 k-steps
template <int L>
__device__ __forceinline__ void load_wt(const h8* lwb, int lane, h8 (&W)[4][2]) {
#pragma unroll
    for (int mb = 0; mb < 4; ++mb)
#pragma unroll
        for (int s = 0; s < 2; ++s) W[mb][s] = lwb[t16_bwd_frag(L, mb, s) * 64 + lane];
}

constexpr int kWaves = 4;  // 4 waves x 2 groups x 16 samples = 128 samples per block

#if NRC_DEBUG_KERNELS  // the 4-wave kernel (round 2, before the role split) and its stamped build
// ABL (diagnostic builds, NRC_T16_ABL): 1 drops the slab stores at compile time, which also drops the dW tiles (dead
// code); 2 keeps the dW tiles and skips only the stores. The product instantiation is ABL = 0.
template <bool STAMP, int ABL = 0>
__global__ __launch_bounds__(256, 1) void train16_kernel(const float* __restrict__ q, const float* __restrict__ t,
                                                         int64_t b, float n_total, float loss_scale,
                                                         const h8* __restrict__ wf, const h8* __restrict__ wb,
                                                         _Float16* __restrict__ slabs, float* __restrict__ loss_partials,
                                                         uint64_t* __restrict__ stamps) {
    const int lane = threadIdx.x & 63;
    int nst = 0;
    // STAMP (diagnostic build only): lane 0 of every wave records s_memtime at 16 phase boundaries into
    // stamps[block][wave][16]
    auto stamp = [&]() {
        if (STAMP) {
            __builtin_amdgcn_sched_barrier(0);
            const uint64_t tt = __builtin_amdgcn_s_memtime();
            __builtin_amdgcn_sched_barrier(0);
            if (lane == 0) stamps[(blockIdx.x * kWaves + (threadIdx.x >> 6)) * 16 + nst] = tt;
            ++nst;
        }
    };
    stamp();
    __shared__ __attribute__((aligned(16))) char smem[kLds];
    h8* lwb = (h8*)(smem + kOffWb);
    h8* lwf = (h8*)(smem + kOffWf);
    char* const img_a0 = smem + kOffImg;
    char* const img_a1 = smem + kOffImg + kImg;
    char* const img_d0 = smem + kOffImg + 2 * kImg;
    char* const img_d1 = smem + kOffImg + 3 * kImg;
    char* const img_x2 = smem + kOffX2;
    float* red = (float*)(smem + kOffRed);

    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int g = lane >> 4, c = lane & 15;
    int r[2];  // image rows (samples within the block) of the wave's two 16-sample groups
    bool valid[2];
    typedef float f3 __attribute__((ext_vector_type(3)));
    f3 pq[2], tq[2];
    f2 bl[2], id[2];
    const int gg = g < 3 ? g : 0;
    // Sample loads by inline asm, so that the compiler does not wait for them itself: it cannot count a
    // vmcnt across the LDS-DMAs issued next and would wait for all of them (vmcnt(0)) before the encoder. The waits
    // are explicit: vmcnt(12) below = the sample loads (issued first) have landed, the 12 DMAs may be in flight.
#pragma unroll
    for (int u = 0; u < 2; ++u) {
        r[u] = 32 * wave + 16 * u + c;
        const int64_t s = (int64_t)blockIdx.x * kTrainSamplesPerBlock + r[u];
        valid[u] = s < b;
        const int64_t sc = valid[u] ? s : b - 1;
        // position, OneBlob dims 3 + 2g, 4 + 2g, Identity dims 9 + 2g, 10 + 2g (lane group 3: dummies with zero
        // weights, fed from group 0's dims so that they stay finite), target
        const float* qr = q + sc * NRC_INPUT_DIMS;
        asm volatile("global_load_dwordx3 %0, %1, off" : "=v"(pq[u]) : "v"(qr) : "memory");
        asm volatile("global_load_dwordx2 %0, %1, off" : "=v"(bl[u]) : "v"(qr + 3 + 2 * gg) : "memory");
        asm volatile("global_load_dwordx2 %0, %1, off" : "=v"(id[u]) : "v"(qr + 9 + 2 * gg) : "memory");
        asm volatile("global_load_dwordx3 %0, %1, off" : "=v"(tq[u]) : "v"(t + sc * 3) : "memory");
    }

    // forward image -> LDS by LDS-DMA (no VGPRs), fragment f from wave f % 4, a fixed 12 per wave in fragment order:
    // per wave, DMAs 0..2 carry layer 0, 3..4 layer 1, 5..6 layer 2, 7..8 layer 3, 9..10 layer 4, 11 layer 5 (the two
    // past the image, 46 and 47, copy fragment 45 into the 2 KiB reserved after it). The forward pass waits layer by
    // layer (vmcnt + barrier), so that only layers 0 and 1 are on its critical path.
    static_assert(kLds >= kOffWf + 12 * kWaves * 1024, "DMA overrun space");
    static_assert(t16_fwd_frag(1, 0, 0) == 3 * kWaves && t16_fwd_frag(2, 0, 0) == 5 * kWaves &&
                      t16_fwd_frag(3, 0, 0) == 7 * kWaves && t16_fwd_frag(4, 0, 0) == 9 * kWaves &&
                      t16_fwd_frag(5, 0, 0) == 11 * kWaves,
                  "layer boundaries fall on DMA rounds");
#pragma unroll
    for (int k = 0; k < 12; ++k) {
        const int f = wave + kWaves * k;
        __builtin_amdgcn_global_load_lds((const void*)(wf + (f < kT16FwdFrags ? f : kT16FwdFrags - 1) * 64 + lane),
                                         (__attribute__((address_space(3))) void*)(lwf + f * 64), 16, 0, 0);
    }

    // the sample loads (their registers are operands, so that no use is scheduled above the wait)
    asm volatile("s_waitcnt vmcnt(12)"
                 : "+v"(pq[0]), "+v"(pq[1]), "+v"(bl[0]), "+v"(bl[1]), "+v"(id[0]), "+v"(id[1]), "+v"(tq[0]), "+v"(tq[1])
                 :
                 : "memory");
    h8 x[2][3];
    float tg[2][3];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
        tg[u][0] = tq[u].x; tg[u][1] = tq[u].y; tg[u][2] = tq[u].z;
        encode16(pq[u].x, pq[u].y, pq[u].z, bl[u].x, bl[u].y, id[u].x, id[u].y, g, x[u]);
        // K slots 64..95 go to their image now (read only by the last step)
        const u4 w = __builtin_bit_cast(u4, x[u][2]);
        *(u2*)(img_x2 + off32(r[u], 2 * g)) = u2{w.x, w.y};
        *(u2*)(img_x2 + off32(r[u], 2 * g + 1)) = u2{w.z, w.w};
    }
    stamp();
    asm volatile("s_waitcnt vmcnt(7)" ::: "memory");  // DMAs 0..4: layers 0 and 1
    lds_barrier();
    stamp();

    // backward image -> LDS by LDS-DMA as well, 9 fragments per wave; it lands during the forward pass (waited for
    // before the barrier after the loss). The forward's later waits count these 9 as younger.
    static_assert(kT16BwdFrags == 9 * kWaves, "backward image tiles the waves");
#pragma unroll
    for (int k = 0; k < 9; ++k) {
        const int f = wave + kWaves * k;
        __builtin_amdgcn_global_load_lds((const void*)(wb + f * 64 + lane),
                                         (__attribute__((address_space(3))) void*)(lwb + f * 64), 16, 0, 0);
    }

    // ---- forward: each A fragment read from LDS feeds both groups' MFMAs. Software-pipelined by hand: a layer's
    // fragments are read while the previous layer computes (the scheduler otherwise issues them two at a time, each
    // pair behind an lgkmcnt(0)).
    h8 a[5][2][2];  // a[l][u][k-step]
    f4 o[2];
    {
        h8 w0[12], w1[8];
#pragma unroll
        for (int mb = 0; mb < 4; ++mb)
#pragma unroll
            for (int ks = 0; ks < 3; ++ks) w0[mb * 3 + ks] = lwf[t16_fwd_frag(0, mb, ks) * 64 + lane];
#pragma unroll
        for (int i = 0; i < 8; ++i) w1[i] = lwf[t16_fwd_frag(1, i >> 1, i & 1) * 64 + lane];
        __builtin_amdgcn_sched_barrier(0);
        f4 cc[2][4];
#pragma unroll
        for (int mb = 0; mb < 4; ++mb) {
            cc[0][mb] = cc[1][mb] = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int ks = 0; ks < 3; ++ks) {
                cc[0][mb] = mfma16(w0[mb * 3 + ks], x[0][ks], cc[0][mb]);
                cc[1][mb] = mfma16(w0[mb * 3 + ks], x[1][ks], cc[1][mb]);
            }
        }
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            a[0][u][0] = relu_b(cc[u][0], cc[u][1]);
            a[0][u][1] = relu_b(cc[u][2], cc[u][3]);
        }
        __builtin_amdgcn_sched_barrier(0);
        stamp();
#pragma unroll
        for (int l = 1; l < 6; ++l) {
            h8 wn[8];  // next layer's fragments (layer 5: 2)
            if (l < 5) {
                // layer l + 1 landed: its DMAs and the 9 backward-image DMAs are younger than what remains
                if (l == 1) asm volatile("s_waitcnt vmcnt(14)" ::: "memory");
                if (l == 2) asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
                if (l == 3) asm volatile("s_waitcnt vmcnt(10)" ::: "memory");
                if (l == 4) asm volatile("s_waitcnt vmcnt(9)" ::: "memory");
                lds_barrier();
#pragma unroll
                for (int i = 0; i < 8; ++i)
                    if (l + 1 < 5 || i < 2) wn[i] = lwf[t16_fwd_frag(l + 1, l + 1 < 5 ? i >> 1 : 0, i & 1) * 64 + lane];
            }
            __builtin_amdgcn_sched_barrier(0);
            if (l < 5) {
#pragma unroll
                for (int mb = 0; mb < 4; ++mb) {
                    cc[0][mb] = cc[1][mb] = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
                    for (int ks = 0; ks < 2; ++ks) {
                        cc[0][mb] = mfma16(w1[mb * 2 + ks], a[l - 1][0][ks], cc[0][mb]);
                        cc[1][mb] = mfma16(w1[mb * 2 + ks], a[l - 1][1][ks], cc[1][mb]);
                    }
                }
#pragma unroll
                for (int u = 0; u < 2; ++u) {
                    a[l][u][0] = relu_b(cc[u][0], cc[u][1]);
                    a[l][u][1] = relu_b(cc[u][2], cc[u][3]);
                }
            } else {
                o[0] = o[1] = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
                for (int ks = 0; ks < 2; ++ks) {
                    o[0] = mfma16(w1[ks], a[4][0][ks], o[0]);
                    o[1] = mfma16(w1[ks], a[4][1][ks], o[1]);
                }
            }
            __builtin_amdgcn_sched_barrier(0);
            stamp();
#pragma unroll
            for (int i = 0; i < 8; ++i) w1[i] = wn[i];
        }
    }

    // ---- RelativeL2Luminance on the f16 prediction (rows 0..2 = registers 0..2 of lane group 0),
    // loss-scaled f16 gradient, ReLU-masked: delta_5 as a 16x16x16 B operand (rows 4g .. 4g + 3). One division per
    // sample (1 / (denom * n_total)) instead of two per channel.
    float lossv = 0.0f;
    h4 d5[2] = {h4{}, h4{}};
    if (g == 0) {
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            float y[3];
#pragma unroll
            for (int k = 0; k < 3; ++k) y[k] = (float)(_Float16)fmaxf(o[u][k], 0.0f);
            const float lum = 0.299f * y[0] + 0.587f * y[1] + 0.114f * y[2];
            const float inv = 1.0f / ((lum * lum + NRC_LUM_EPS) * n_total);
#pragma unroll
            for (int k = 0; k < 3; ++k) {
                const float diff = y[k] - tg[u][k];
                lossv += valid[u] ? diff * diff * inv : 0.0f;
                d5[u][k] = (valid[u] && y[k] > 0.0f) ? (_Float16)(loss_scale * 2.0f * diff * inv) : (_Float16)0.0f;
            }
        }
    }
    lossv = row_sum16(lossv);  // lane group 0 = row 0 holds every nonzero term
    if (lane == 0) red[wave] = lossv;

    _Float16* slab = slabs + (int64_t)blockIdx.x * slab_floats(0);
    // ABL 2 (diagnostic): the slab stores sit behind a run-time condition that is never true (loss_scale < 0), so the
    // dW tiles are still computed but nothing is stored
    const bool do_store = !(ABL & 2) || loss_scale < 0.0f;

    // image-row write offsets of the two groups, kept for the whole backward pass
    int wo[2][4];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
        row_offsets(r[u], g, wo[u]);
        asm volatile("" : "+v"(wo[u][0]), "+v"(wo[u][1]), "+v"(wo[u][2]), "+v"(wo[u][3]));
    }
    // layer-5 operands (buffer 1): delta_5 rows 4g .. 4g + 3 = quad g, a_4
#pragma unroll
    for (int u = 0; u < 2; ++u) {
        *(h4*)(img_d1 + off64(r[u], g)) = d5[u];
        put_rows64(img_a1, wo[u], a[4][u]);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // backward image landed
    lds_barrier();
    if (threadIdx.x == 0) {
        const float lp = (red[0] + red[1]) + (red[2] + red[3]);
        loss_partials[blockIdx.x] = lp;
    }
    stamp();

    // transposed-read tiles of this wave: dW rows tm = 2 (wave >> 1) + i, columns tn = 2 (wave & 1) + j
    const int G = lane >> 4, qq = (lane >> 2) & 3, pp = lane & 3;
    const int r0 = 8 * G + qq, r1 = r0 + 4;
    const int tm0 = 2 * (wave >> 1), tn0 = 2 * (wave & 1);
    int oa[2][2], ob[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        oa[i][0] = off64(r0, 4 * (tm0 + i) + pp);
        oa[i][1] = off64(r1, 4 * (tm0 + i) + pp);
        ob[i][0] = off64(r0, 4 * (tn0 + i) + pp);
        ob[i][1] = off64(r1, 4 * (tn0 + i) + pp);
        asm volatile("" : "+v"(oa[i][0]), "+v"(oa[i][1]), "+v"(ob[i][0]), "+v"(ob[i][1]));
    }
    auto tiles = [&](const char* imgd, const char* imga, TrTile (&ta)[2], TrTile (&tb)[2]) {
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            ta[i] = TrTile{imgd, oa[i][0], oa[i][1], 4096};
            tb[i] = TrTile{imga, ob[i][0], ob[i][1], 4096};
        }
    };
    // Slab stores are deferred by one step: a step stores the previous step's two tile pairs (dW rows tm0, tm0 + 1)
    // from its first two MFMA phases, so that the stored values are never waiting on MFMAs.
    u4 pend[2];
    int pend_L = -1;
    auto flush = [&](int i) {
        if constexpr (!(ABL & 1))
            if (pend_L >= 0 && do_store) slab_pair(slab, pend_L, tm0 + i, tn0, lane, pend[i]);
    };

    h8 d[2][2], dn[2][2], W[4][2];
    // ---- step 5 (buffer 1): dW5 tile (0, wave); delta_4 = W5^T delta_5 * [a_4 > 0] (16x16x16: K = 16 output rows)
    {
        const h4* lwb4 = (const h4*)lwb;
        h4 W5[4];
#pragma unroll
        for (int mb = 0; mb < 4; ++mb) W5[mb] = lwb4[t16_bwd_frag(5, mb, 0) * 128 + lane];
        f4 acc[1][1];
        {
            const TrTile ta[1] = {TrTile{img_d1, off64(r0, pp), off64(r1, pp), 4096}};
            const TrTile tb[1] = {TrTile{img_a1, off64(r0, 4 * wave + pp), off64(r1, 4 * wave + pp), 4096}};
            dw_tiles<1, 1>(ta, tb, acc);
        }
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            f4 cc[4];
#pragma unroll
            for (int mb = 0; mb < 4; ++mb) cc[mb] = mfma16k16(W5[mb], d5[u], f4{0.f, 0.f, 0.f, 0.f});
#pragma unroll
            for (int s2 = 0; s2 < 2; ++s2) d[u][s2] = gate_b(cc[2 * s2], cc[2 * s2 + 1], a[4][u][s2]);
            put_rows64(img_d0, wo[u], d[u]);
            put_rows64(img_a0, wo[u], a[3][u]);
        }
        if constexpr (!(ABL & 1))
            if (do_store) slab_single(slab, 5, 0, wave, lane, acc[0][0]);
        load_wt<4>(lwb, lane, W);
    }
    lds_barrier();
    stamp();

    // ---- steps 4..1: dW_L from buffer L & 1, delta_{L-1} into the other buffer with a_{L-2} (step 1: the input
    // slots 0..63, quads 8s + 2g, 8s + 2g + 1). Phases fenced by sched_barrier: the dW operand reads and the a_{L-2}
    // writes; the chain's MFMAs of group 0, then group 1 (each with one deferred slab store); the next layer's W^T
    // reads; the dW tiles of row 0 with group 0's gate and delta writes, then row 1 with group 1's.
#define NRC_T16_STEP(L, IMGD, IMGA, NIMGD, NIMGA)                                                                  \
    {                                                                                                              \
        TrTile ta[2], tb[2];                                                                                       \
        tiles(IMGD, IMGA, ta, tb);                                                                                 \
        h8 A[2][4], B[2][4];                                                                                       \
        _Pragma("unroll") for (int i = 0; i < 2; ++i) _Pragma("unroll") for (int kk = 0; kk < 4; ++kk) {           \
            A[i][kk] = tr_op(ta[i], kk);                                                                           \
            B[i][kk] = tr_op(tb[i], kk);                                                                           \
        }                                                                                                          \
        /* a_{L-2} (step 1: the input slots 0..63) does not depend on this step: written first */                  \
        _Pragma("unroll") for (int u = 0; u < 2; ++u) {                                                            \
            if constexpr (L > 1) {                                                                                 \
                put_rows64(NIMGA, wo[u], a[L > 1 ? L - 2 : 0][u]);                                                 \
            } else {                                                                                               \
                _Pragma("unroll") for (int ks = 0; ks < 2; ++ks) {                                                 \
                    const u4 w = __builtin_bit_cast(u4, x[u][ks]);                                                 \
                    *(u2*)(NIMGA + off64(r[u], 8 * ks + 2 * g)) = u2{w.x, w.y};                                    \
                    *(u2*)(NIMGA + off64(r[u], 8 * ks + 2 * g + 1)) = u2{w.z, w.w};                                \
                }                                                                                                  \
            }                                                                                                      \
        }                                                                                                          \
        __builtin_amdgcn_sched_barrier(0);                                                                         \
        f4 cc[2][4];                                                                                               \
        _Pragma("unroll") for (int u = 0; u < 2; ++u) {                                                            \
            _Pragma("unroll") for (int mb = 0; mb < 4; ++mb) {                                                     \
                cc[u][mb] = mfma16(W[mb][0], d[u][0], f4{0.f, 0.f, 0.f, 0.f});                                     \
                cc[u][mb] = mfma16(W[mb][1], d[u][1], cc[u][mb]);                                                  \
            }                                                                                                      \
            flush(u);                                                                                              \
            __builtin_amdgcn_sched_barrier(0);                                                                     \
        }                                                                                                          \
        /* W is dead after the chain: the next layer's W^T reads go out with the first dW half */                  \
        if constexpr (L > 1) load_wt<(L > 1 ? L - 1 : 1)>(lwb, lane, W);                                            \
        f4 acc[2][2];                                                                                              \
        _Pragma("unroll") for (int i = 0; i < 2; ++i) {                                                            \
            _Pragma("unroll") for (int j = 0; j < 2; ++j) {                                                        \
                acc[i][j] = f4{0.f, 0.f, 0.f, 0.f};                                                                \
                _Pragma("unroll") for (int kk = 0; kk < 4; ++kk) acc[i][j] = mfma16(A[i][kk], B[j][kk], acc[i][j]); \
            }                                                                                                      \
            _Pragma("unroll") for (int s2 = 0; s2 < 2; ++s2)                                                       \
                dn[i][s2] = gate_b(cc[i][2 * s2], cc[i][2 * s2 + 1], a[L - 1][i][s2]);                             \
            put_rows64(NIMGD, wo[i], dn[i]);                                                                       \
            __builtin_amdgcn_sched_barrier(0);                                                                     \
        }                                                                                                          \
        _Pragma("unroll") for (int i = 0; i < 2; ++i) pend[i] = pack_pair(acc[i][0], acc[i][1]);                    \
        pend_L = L;                                                                                                \
        _Pragma("unroll") for (int u = 0; u < 2; ++u)                                                              \
            _Pragma("unroll") for (int s2 = 0; s2 < 2; ++s2) d[u][s2] = dn[u][s2];                                 \
    }                                                                                                              \
    lds_barrier();                                                                                                 \
    stamp();
    NRC_T16_STEP(4, img_d0, img_a0, img_d1, img_a1)
    NRC_T16_STEP(3, img_d1, img_a1, img_d0, img_a0)
    NRC_T16_STEP(2, img_d0, img_a0, img_d1, img_a1)
    NRC_T16_STEP(1, img_d1, img_a1, img_d0, img_a0)
#undef NRC_T16_STEP
    // ---- step 0 (buffer 0): dW0 tiles (tm0 + i, 3 (wave & 1) + j); columns 4, 5 are K slots 64..95 (img_x2)
    {
        f4 acc[2][3];
        const TrTile ta[2] = {TrTile{img_d0, oa[0][0], oa[0][1], 4096}, TrTile{img_d0, oa[1][0], oa[1][1], 4096}};
        if ((wave & 1) == 0) {
            const TrTile tb[3] = {TrTile{img_a0, off64(r0, pp), off64(r1, pp), 4096},
                                  TrTile{img_a0, off64(r0, 4 + pp), off64(r1, 4 + pp), 4096},
                                  TrTile{img_a0, off64(r0, 8 + pp), off64(r1, 8 + pp), 4096}};
            dw_tiles<2, 3>(ta, tb, acc);
        } else {
            const TrTile tb[3] = {TrTile{img_a0, off64(r0, 12 + pp), off64(r1, 12 + pp), 4096},
                                  TrTile{img_x2, off32(r0, pp), off32(r1, pp), 2048},
                                  TrTile{img_x2, off32(r0, 4 + pp), off32(r1, 4 + pp), 2048}};
            dw_tiles<2, 3>(ta, tb, acc);
        }
        flush(0);
        flush(1);
        if (!(ABL & 1) && do_store) {
#pragma unroll
            for (int i = 0; i < 2; ++i) {
                if ((wave & 1) == 0) {  // tiles 0, 1 (a pair) and 2 (the even half of pair 2, 3)
                    slab_pair(slab, 0, tm0 + i, 0, lane, pack_pair(acc[i][0], acc[i][1]));
                    slab_single(slab, 0, tm0 + i, 2, lane, acc[i][2]);
                } else {  // tile 3 (the odd half of pair 2, 3) and tiles 4, 5
                    slab_single(slab, 0, tm0 + i, 3, lane, acc[i][0]);
                    slab_pair(slab, 0, tm0 + i, 4, lane, pack_pair(acc[i][1], acc[i][2]));
                }
            }
        }
    }
    stamp();
}

#endif

// Role-split variant (NRC_T16_SPLIT, A/B): 8 waves per block, 2 per SIMD. Waves 0..3 ("chain") do what
// train16_kernel's waves do except the weight gradients: encode, forward, loss, then per backward step the delta chain
// (W_L^T delta_L, ReLU gate) and the image writes. Waves 4..7 ("dW") sit through the forward at its barriers and then,
// in each backward step, compute the block's dW_L tiles from the images the chain waves wrote in the step before and
// stream them to the slab. The two halves of a step share the SIMDs' MFMA pipes and hide each other's LDS and
// dependency latency; the step's critical path is the chain alone instead of chain + dW.
// G: 16-sample groups per chain wave (64 G samples per block); PADQ: padded RadianceQuery records (16 floats: the
// position load takes pad_ along, 16 bytes instead of 12, the other loads one float further)
// ENC 3 / 1 (round 5): InputEncoding::Hash -- the encoder reads each lane group's 4 grid levels (t16_hash_slot_feature)
// from the batch's feature pass (3) or gathers them from the table (1, A/B),
// and after the last chain step the chain waves form dL/d(grid features) = W0^T delta_0 (4 MFMAs per group from the
// backward image's fragments 36..39, read from global memory) and write it with the sample positions for
// grid_scatter_kernel (ho). Everything else -- forward, loss, delta chain, dW waves, slab layout -- is the Frequency
// kernel's.
// The body takes the block's LDS and index from its kernel (train16_split_kernel, or the fused step's trainer blocks).
// PRIO (debug library, A/B): 1 = the dW waves at s_setprio 1, 2 = the chain waves at s_setprio 1 (issue arbitration
// is by priority, then age; the chain waves are the older half)
template <int AUX, int G = 2, bool PADQ = false, int ENC = 0, int PRIO = 0>
__device__ __forceinline__ void train16_split_body(char* __restrict__ smem, const int blk,
                                                   const float* __restrict__ q, const float* __restrict__ t, int64_t b,
                                                   float n_total, float loss_scale, const h8* __restrict__ wf,
                                                   const h8* __restrict__ wb, _Float16* __restrict__ slabs,
                                                   float* __restrict__ loss_partials, const HashTrainOut& ho) {
    const int lane = threadIdx.x & 63;
    h8* lwb = (h8*)(smem + kOffWb);
    h8* lwf = (h8*)(smem + kOffWf);
    char* const img_a0 = smem + kOffImg;
    char* const img_a1 = smem + kOffImg + kImg;
    char* const img_d0 = smem + kOffImg + 2 * kImg;
    char* const img_d1 = smem + kOffImg + 3 * kImg;
    char* const img_x2 = smem + kOffX2;
    float* red = (float*)(smem + kOffRed);
    const int wave_all = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const bool dw_wave = wave_all >= kWaves;
    const int wave = dw_wave ? wave_all - kWaves : wave_all;
    const int g = lane >> 4, c = lane & 15;
    _Float16* slab = slabs + (int64_t)blk * slab_floats(0);

    if (dw_wave) {
        if constexpr (PRIO == 1) __builtin_amdgcn_s_setprio(1);
        // ---- dW waves: the forward's six barriers, then one dW step per backward step
        for (int i = 0; i < 6; ++i) lds_barrier();
        const int lg = lane >> 4, qq = (lane >> 2) & 3, pp = lane & 3;
        const int r0 = 8 * lg + qq, r1 = r0 + 4;
        const int tm0 = 2 * (wave >> 1), tn0 = 2 * (wave & 1);
        int oa[2][2], ob[2][2];
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            oa[i][0] = off64(r0, 4 * (tm0 + i) + pp);
            oa[i][1] = off64(r1, 4 * (tm0 + i) + pp);
            ob[i][0] = off64(r0, 4 * (tn0 + i) + pp);
            ob[i][1] = off64(r1, 4 * (tn0 + i) + pp);
        }
        // step 5 (buffer 1): dW5 tile (0, wave)
        {
            f4 acc[1][1];
            const TrTile ta[1] = {TrTile{img_d1, off64(r0, pp), off64(r1, pp), 4096}};
            const TrTile tb[1] = {TrTile{img_a1, off64(r0, 4 * wave + pp), off64(r1, 4 * wave + pp), 4096}};
            dw_tiles<1, 1, 2 * G>(ta, tb, acc);
            slab_single_b<AUX>(slab, 5, 0, wave, lane, acc[0][0]);
        }
        lds_barrier();
        // steps 4..1: dW_L tiles (tm0 + i, tn0 + j) from buffer L & 1
#pragma unroll
        for (int L = 4; L >= 1; --L) {
            const char* imgd = (L & 1) ? img_d1 : img_d0;
            const char* imga = (L & 1) ? img_a1 : img_a0;
            TrTile ta[2], tb[2];
#pragma unroll
            for (int i = 0; i < 2; ++i) {
                ta[i] = TrTile{imgd, oa[i][0], oa[i][1], 4096};
                tb[i] = TrTile{imga, ob[i][0], ob[i][1], 4096};
            }
            f4 acc[2][2];
            dw_tiles<2, 2, 2 * G>(ta, tb, acc);
#pragma unroll
            for (int i = 0; i < 2; ++i) slab_pair_b<AUX>(slab, L, tm0 + i, tn0, lane, pack_pair(acc[i][0], acc[i][1]));
            lds_barrier();
        }
        // step 0 (buffer 0): dW0 tiles (tm0 + i, 3 (wave & 1) + j); columns 4, 5 are K slots 64..95 (img_x2)
        {
            f4 acc[2][3];
            const TrTile ta[2] = {TrTile{img_d0, oa[0][0], oa[0][1], 4096}, TrTile{img_d0, oa[1][0], oa[1][1], 4096}};
            if ((wave & 1) == 0) {
                const TrTile tb[3] = {TrTile{img_a0, off64(r0, pp), off64(r1, pp), 4096},
                                      TrTile{img_a0, off64(r0, 4 + pp), off64(r1, 4 + pp), 4096},
                                      TrTile{img_a0, off64(r0, 8 + pp), off64(r1, 8 + pp), 4096}};
                dw_tiles<2, 3, 2 * G>(ta, tb, acc);
            } else {
                const TrTile tb[3] = {TrTile{img_a0, off64(r0, 12 + pp), off64(r1, 12 + pp), 4096},
                                      TrTile{img_x2, off32(r0, pp), off32(r1, pp), 2048},
                                      TrTile{img_x2, off32(r0, 4 + pp), off32(r1, 4 + pp), 2048}};
                dw_tiles<2, 3, 2 * G>(ta, tb, acc);
            }
#pragma unroll
            for (int i = 0; i < 2; ++i) {
                if ((wave & 1) == 0) {
                    slab_pair_b<AUX>(slab, 0, tm0 + i, 0, lane, pack_pair(acc[i][0], acc[i][1]));
                    slab_single_b<AUX>(slab, 0, tm0 + i, 2, lane, acc[i][2]);
                } else {
                    slab_single_b<AUX>(slab, 0, tm0 + i, 3, lane, acc[i][0]);
                    slab_pair_b<AUX>(slab, 0, tm0 + i, 4, lane, pack_pair(acc[i][1], acc[i][2]));
                }
            }
        }
        return;
    }

    // ---- chain waves: as train16_kernel
    if constexpr (PRIO == 2) __builtin_amdgcn_s_setprio(1);
    int r[G];
    bool valid[G];
    typedef float f3 __attribute__((ext_vector_type(3)));
    typedef float f4v __attribute__((ext_vector_type(4)));
    typedef std::conditional_t<PADQ, f4v, f3> PQ;
    constexpr int X = PADQ ? 1 : 0;
    PQ pq[G];
    f3 tq[G];
    f2 bl[G], id[G];
    [[maybe_unused]] uint32_t F[G][4];  // ENC 3: the sample's level features 4g .. 4g + 3 (hash_feature_kernel)
    const int gg = g < 3 ? g : 0;
#pragma unroll
    for (int u = 0; u < G; ++u) {
        r[u] = 16 * (G * wave + u) + c;
        const int64_t s = (int64_t)blk * (64 * G) + r[u];
        valid[u] = s < b;
        const int64_t sc = valid[u] ? s : b - 1;
        const float* qr = q + sc * (NRC_INPUT_DIMS + X);
        if constexpr (PADQ) asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(pq[u]) : "v"(qr) : "memory");
        else asm volatile("global_load_dwordx3 %0, %1, off" : "=v"(pq[u]) : "v"(qr) : "memory");
        asm volatile("global_load_dwordx2 %0, %1, off" : "=v"(bl[u]) : "v"(qr + 3 + X + 2 * gg) : "memory");
        asm volatile("global_load_dwordx2 %0, %1, off" : "=v"(id[u]) : "v"(qr + 9 + X + 2 * gg) : "memory");
        asm volatile("global_load_dwordx3 %0, %1, off" : "=v"(tq[u]) : "v"(t + sc * 3) : "memory");
        if constexpr (ENC == 3) {
            // padding samples read the last sample's features (finite), as they read its query
            const uint32_t* fr = ho.feat + (int64_t)(4 * g) * kHashFeatStride + sc;
#pragma unroll
            for (int i = 0; i < 4; ++i)
                asm volatile("global_load_dword %0, %1, off" : "=v"(F[u][i]) : "v"(fr + i * kHashFeatStride) : "memory");
        }
    }
#pragma unroll
    for (int k = 0; k < 12; ++k) {
        const int f = wave + kWaves * k;
        __builtin_amdgcn_global_load_lds((const void*)(wf + (f < kT16FwdFrags ? f : kT16FwdFrags - 1) * 64 + lane),
                                         (__attribute__((address_space(3))) void*)(lwf + f * 64), 16, 0, 0);
    }
    if constexpr (G == 2 && ENC == 3)
        asm volatile("s_waitcnt vmcnt(12)"
                     : "+v"(pq[0]), "+v"(pq[1]), "+v"(bl[0]), "+v"(bl[1]), "+v"(id[0]), "+v"(id[1]), "+v"(tq[0]), "+v"(tq[1]),
                       "+v"(F[0][0]), "+v"(F[0][1]), "+v"(F[0][2]), "+v"(F[0][3]), "+v"(F[1][0]), "+v"(F[1][1]),
                       "+v"(F[1][2]), "+v"(F[1][3])
                     :
                     : "memory");
    else if constexpr (G == 2)
        asm volatile("s_waitcnt vmcnt(12)"
                     : "+v"(pq[0]), "+v"(pq[1]), "+v"(bl[0]), "+v"(bl[1]), "+v"(id[0]), "+v"(id[1]), "+v"(tq[0]), "+v"(tq[1])
                     :
                     : "memory");
    else
        asm volatile("s_waitcnt vmcnt(12)" : "+v"(pq[0]), "+v"(bl[0]), "+v"(id[0]), "+v"(tq[0]) : : "memory");
    h8 x[G][3];
    float tg[G][3];
#pragma unroll
    for (int u = 0; u < G; ++u) {
        tg[u][0] = tq[u].x; tg[u][1] = tq[u].y; tg[u][2] = tq[u].z;
        float pad = 1.0f;
        if constexpr (PADQ) pad = pq[u].w;
        if constexpr (ENC == 3) encode16_hashf(F[u], bl[u].x, bl[u].y, id[u].x, id[u].y, g, x[u], pad);
        else if constexpr (ENC == 1) encode16_hash(pq[u].x, pq[u].y, pq[u].z, bl[u].x, bl[u].y, id[u].x, id[u].y, g, ho.table, x[u], pad);
        else encode16(pq[u].x, pq[u].y, pq[u].z, bl[u].x, bl[u].y, id[u].x, id[u].y, g, x[u], pad);
        const u4 w = __builtin_bit_cast(u4, x[u][2]);
        *(u2*)(img_x2 + off32(r[u], 2 * g)) = u2{w.x, w.y};
        *(u2*)(img_x2 + off32(r[u], 2 * g + 1)) = u2{w.z, w.w};
    }
    asm volatile("s_waitcnt vmcnt(7)" ::: "memory");
    lds_barrier();  // barrier 1
#pragma unroll
    for (int k = 0; k < 9; ++k) {
        const int f = wave + kWaves * k;
        __builtin_amdgcn_global_load_lds((const void*)(wb + f * 64 + lane),
                                         (__attribute__((address_space(3))) void*)(lwb + f * 64), 16, 0, 0);
    }
    h8 a[5][G][2];
    f4 o[G];
    {
        h8 w0[12], w1[8];
#pragma unroll
        for (int mb = 0; mb < 4; ++mb)
#pragma unroll
            for (int ks = 0; ks < 3; ++ks) w0[mb * 3 + ks] = lwf[t16_fwd_frag(0, mb, ks) * 64 + lane];
#pragma unroll
        for (int i = 0; i < 8; ++i) w1[i] = lwf[t16_fwd_frag(1, i >> 1, i & 1) * 64 + lane];
        __builtin_amdgcn_sched_barrier(0);
        f4 cc[G][4];
#pragma unroll
        for (int mb = 0; mb < 4; ++mb) {
#pragma unroll
            for (int u = 0; u < G; ++u) cc[u][mb] = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int ks = 0; ks < 3; ++ks)
#pragma unroll
                for (int u = 0; u < G; ++u) cc[u][mb] = mfma16(w0[mb * 3 + ks], x[u][ks], cc[u][mb]);
        }
#pragma unroll
        for (int u = 0; u < G; ++u) {
            a[0][u][0] = relu_b(cc[u][0], cc[u][1]);
            a[0][u][1] = relu_b(cc[u][2], cc[u][3]);
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int l = 1; l < 6; ++l) {
            h8 wn[8];
            if (l < 5) {
                if (l == 1) asm volatile("s_waitcnt vmcnt(14)" ::: "memory");
                if (l == 2) asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
                if (l == 3) asm volatile("s_waitcnt vmcnt(10)" ::: "memory");
                if (l == 4) asm volatile("s_waitcnt vmcnt(9)" ::: "memory");
                lds_barrier();  // barriers 2..5
#pragma unroll
                for (int i = 0; i < 8; ++i)
                    if (l + 1 < 5 || i < 2) wn[i] = lwf[t16_fwd_frag(l + 1, l + 1 < 5 ? i >> 1 : 0, i & 1) * 64 + lane];
            }
            __builtin_amdgcn_sched_barrier(0);
            if (l < 5) {
#pragma unroll
                for (int mb = 0; mb < 4; ++mb) {
#pragma unroll
                    for (int u = 0; u < G; ++u) cc[u][mb] = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
                    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
                        for (int u = 0; u < G; ++u) cc[u][mb] = mfma16(w1[mb * 2 + ks], a[l - 1][u][ks], cc[u][mb]);
                }
#pragma unroll
                for (int u = 0; u < G; ++u) {
                    a[l][u][0] = relu_b(cc[u][0], cc[u][1]);
                    a[l][u][1] = relu_b(cc[u][2], cc[u][3]);
                }
            } else {
#pragma unroll
                for (int u = 0; u < G; ++u) o[u] = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
                for (int ks = 0; ks < 2; ++ks)
#pragma unroll
                    for (int u = 0; u < G; ++u) o[u] = mfma16(w1[ks], a[4][u][ks], o[u]);
            }
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int i = 0; i < 8; ++i) w1[i] = wn[i];
        }
    }
    float lossv = 0.0f;
    h4 d5[G];
#pragma unroll
    for (int u = 0; u < G; ++u) d5[u] = h4{};
    if (g == 0) {
#pragma unroll
        for (int u = 0; u < G; ++u) {
            float y[3];
#pragma unroll
            for (int k = 0; k < 3; ++k) y[k] = (float)(_Float16)fmaxf(o[u][k], 0.0f);
            const float lum = 0.299f * y[0] + 0.587f * y[1] + 0.114f * y[2];
            const float inv = 1.0f / ((lum * lum + NRC_LUM_EPS) * n_total);
#pragma unroll
            for (int k = 0; k < 3; ++k) {
                const float diff = y[k] - tg[u][k];
                lossv += valid[u] ? diff * diff * inv : 0.0f;
                d5[u][k] = (valid[u] && y[k] > 0.0f) ? (_Float16)(loss_scale * 2.0f * diff * inv) : (_Float16)0.0f;
            }
        }
    }
    lossv = row_sum16(lossv);
    if (lane == 0) red[wave] = lossv;
    int wo[G][4];
#pragma unroll
    for (int u = 0; u < G; ++u) {
        row_offsets(r[u], g, wo[u]);
        asm volatile("" : "+v"(wo[u][0]), "+v"(wo[u][1]), "+v"(wo[u][2]), "+v"(wo[u][3]));
    }
#pragma unroll
    for (int u = 0; u < G; ++u) {
        *(h4*)(img_d1 + off64(r[u], g)) = d5[u];
        put_rows64(img_a1, wo[u], a[4][u]);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // backward image landed
    lds_barrier();  // barrier 6
    if (threadIdx.x == 0) {
        const float lp = (red[0] + red[1]) + (red[2] + red[3]);
        // an agent-scope store (sc1): the fused step's reducers on other XCDs read it in the same launch
        __hip_atomic_store(loss_partials + blk, lp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }

    h8 d[G][2], dn[G][2], W[4][2];
    // step 5: delta_4 = W5^T delta_5 * [a_4 > 0] (16x16x16: K = 16 output rows) into buffer 0 with a_3
    {
        const h4* lwb4 = (const h4*)lwb;
        h4 W5[4];
#pragma unroll
        for (int mb = 0; mb < 4; ++mb) W5[mb] = lwb4[t16_bwd_frag(5, mb, 0) * 128 + lane];
#pragma unroll
        for (int u = 0; u < G; ++u) {
            f4 cc[4];
#pragma unroll
            for (int mb = 0; mb < 4; ++mb) cc[mb] = mfma16k16(W5[mb], d5[u], f4{0.f, 0.f, 0.f, 0.f});
#pragma unroll
            for (int s2 = 0; s2 < 2; ++s2) d[u][s2] = gate_b(cc[2 * s2], cc[2 * s2 + 1], a[4][u][s2]);
            put_rows64(img_d0, wo[u], d[u]);
            put_rows64(img_a0, wo[u], a[3][u]);
        }
        load_wt<4>(lwb, lane, W);
    }
    lds_barrier();
    // steps 4..1: delta_{L-1} into the other buffer with a_{L-2} (step 1: the input slots 0..63)
#define NRC_T16S_STEP(L, NIMGD, NIMGA)                                                                              \
    {                                                                                                              \
        _Pragma("unroll") for (int u = 0; u < G; ++u) {                                                            \
            if constexpr (L > 1) {                                                                                 \
                put_rows64(NIMGA, wo[u], a[L > 1 ? L - 2 : 0][u]);                                                 \
            } else {                                                                                               \
                _Pragma("unroll") for (int ks = 0; ks < 2; ++ks) {                                                 \
                    const u4 w = __builtin_bit_cast(u4, x[u][ks]);                                                 \
                    *(u2*)(NIMGA + off64(r[u], 8 * ks + 2 * g)) = u2{w.x, w.y};                                    \
                    *(u2*)(NIMGA + off64(r[u], 8 * ks + 2 * g + 1)) = u2{w.z, w.w};                                \
                }                                                                                                  \
            }                                                                                                      \
        }                                                                                                          \
        chain_groups<G>(W, d, a[L - 1], dn);                                                                                \
        if constexpr (L > 1) load_wt<(L > 1 ? L - 1 : 1)>(lwb, lane, W);                                           \
        _Pragma("unroll") for (int u = 0; u < G; ++u) {                                                            \
            put_rows64(NIMGD, wo[u], dn[u]);                                                                       \
            _Pragma("unroll") for (int s2 = 0; s2 < 2; ++s2) d[u][s2] = dn[u][s2];                                 \
        }                                                                                                          \
    }                                                                                                              \
    lds_barrier();
    // Hash: W0^T of the grid features (16x16x32 A operands, fragments 36 + 2 mb + s), loaded from global memory during
    // the chain (they are read once, after the last step)
    [[maybe_unused]] h8 W0g[2][2];
    if constexpr (ENC == 1 || ENC == 3) {
#pragma unroll
        for (int mb = 0; mb < 2; ++mb)
#pragma unroll
            for (int s = 0; s < 2; ++s) W0g[mb][s] = wb[(kT16BwdFrags + 2 * mb + s) * 64 + lane];
    }
    NRC_T16S_STEP(4, img_d1, img_a1)
    NRC_T16S_STEP(3, img_d0, img_a0)
    NRC_T16S_STEP(2, img_d1, img_a1)
    NRC_T16S_STEP(1, img_d0, img_a0)
#undef NRC_T16S_STEP
    if constexpr (ENC == 1 || ENC == 3) {
        // dL/d(grid slot 16 mb + 4 g + i) of sample c = (W0^T delta_0): registers (0, 1) / (2, 3) of M-block mb are the
        // two features of levels 8 mb + 2 g and 8 mb + 2 g + 1; f16 pairs [level][sample], zeros for padding samples
#pragma unroll
        for (int u = 0; u < G; ++u) {
            const int64_t sg = (int64_t)blk * (64 * G) + r[u];
#pragma unroll
            for (int mb = 0; mb < 2; ++mb) {
                f4 c = mfma16(W0g[mb][0], d[u][0], f4{0.f, 0.f, 0.f, 0.f});
                c = mfma16(W0g[mb][1], d[u][1], c);
                const int lv = 8 * mb + 2 * g;
                ho.dy[(int64_t)lv * ho.bcap + sg] = valid[u] ? pk2(c[0], c[1]) : 0u;
                ho.dy[(int64_t)(lv + 1) * ho.bcap + sg] = valid[u] ? pk2(c[2], c[3]) : 0u;
            }
            if (g == 0) ho.pos[sg] = float4{pq[u].x, pq[u].y, pq[u].z, 0.0f};
        }
    }
}

template <int AUX, int G = 2, bool PADQ = false, int ENC = 0, int PRIO = 0>
__global__ __launch_bounds__(512, 1) void train16_split_kernel(const float* __restrict__ q, const float* __restrict__ t,
                                                               int64_t b, float n_total, float loss_scale,
                                                               const h8* __restrict__ wf, const h8* __restrict__ wb,
                                                               _Float16* __restrict__ slabs,
                                                               float* __restrict__ loss_partials, HashTrainOut ho) {
    __shared__ __attribute__((aligned(16))) char smem[kLds];
    train16_split_body<AUX, G, PADQ, ENC, PRIO>(smem, blockIdx.x, q, t, b, n_total, loss_scale, wf, wb, slabs,
                                                loss_partials, ho);
}

// ---- Round 6: the whole Frequency training step in one launch ----------------------------------
// The step was two launches back to back: train16_split_kernel (128 blocks of 128 samples, one per CU: half the chip idle)
// and reduce_adam_kernel (the fixed-order slab sums + Adam/EMA), and the second paid a kernel boundary and its own ramp
// after the first had ended. Here the first ntrain blocks of one grid are the training kernel's blocks and the next nred
// blocks are reducers: dispatched after every trainer block (workgroups dispatch in order), they land on the idle CUs
// (a block holds a whole CU's LDS, so a reducer never shares a trainer's CU), load their parameters' Adam state, and wait
// until every trainer wave has counted itself in. Each trainer wave counts in after s_waitcnt vmcnt(0): its slab and loss
// stores have completed, and they are agent-scope (sc1) stores, so every reducer on any XCD reads them with agent-scope
// loads (the memory model's relaxed atomics: coherent across the XCDs' L2s, no cache writeback or invalidate). A reducer then sums the slabs and applies Adam/EMA with exactly the float
// operations of reduce_adam_kernel (kReduceFused): 64-position chunks, 16 slab groups of 16 position quads, element k of
// a group's sequence into a0 / a1 by parity, the 16 groups combined in the same tree; the state is bitwise that of the
// two-launch step. Reducer rb takes chunks rb, rb + nred, rb + 2 nred (threads 256..511 the middle one), all loads in
// flight at once. The last reducer past the wait zeroes both counters for the next launch (stream order), so there is no
// host-side generation and a captured graph replays correctly. The wait is bounded (error word 3 -> NRC_ERR_INTERNAL).
constexpr int kFuseChunksPerReducer = 3;
struct FuseArgs {
    ModelBuffers mb;
    OptimArgs oa;
    float lr_t, ema_debias;
    float* loss_out;
    uint32_t* sync;  // [0] trainer waves counted in, [64] reducers past the wait (uncached; 0 between launches)
    uint32_t* err;
    int polls, ntrain, nred, nchunks;
    int mode;      // A/B (knob fuse_mode): 0 flags (default), 1 counter arrival per block, 2 counter per wave
    uint32_t gen;  // mode 0: this launch's generation (host counter, never 0): trainer block i stores it to flags[i]
    uint32_t* flags;
};

__device__ __forceinline__ void fuse_reduce(char* __restrict__ smem, const int rb, const _Float16* __restrict__ slabs,
                                            const float* __restrict__ loss_partials, const FuseArgs& fa) {
#pragma clang fp contract(off)
    const ModelBuffers& mb = fa.mb;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    if (fa.mode == 3) return;  // timing ablation (wrong results): no reducers
    const int nslabs = fa.ntrain;
    // Adam state of the parameter this lane applies (waves 0..2: chunk rb + wave nred, position lane), loaded first
    const int ach = rb + wave * fa.nred;
    const int pp = (wave < kFuseChunksPerReducer && ach < fa.nchunks) ? t16_slab_param(ach * 64 + lane) : -1;
    AdamIn ain{};
    if (pp >= 0) ain = adam_load(pp, mb);
    asm volatile("" : "+v"(ain.fp), "+v"(ain.ft), "+v"(ain.bp));
    // the wait: wave 0 polls, the block follows at the barrier. Mode 0: every trainer block's flag holds this launch's
    // generation (lane l reads flags l, l + 64, ...; agent-scope loads, no read-modify-write anywhere). Modes 1 / 2 (A/B):
    // an arrival counter that trainer blocks / waves increment and the last reducer resets -- each atomic on the one
    // word costs ~14 ns serialised (1,024 per-wave arrivals: 27.8 us per step, 128 per-block: 15.2 us, round 6 A/B)
    if (wave == 0 && (fa.mode == 0 || fa.mode == 4)) {
        int i = 0;
        for (; i < fa.polls; ++i) {
            bool ok = true;
            for (int k = lane; k < fa.ntrain; k += 64)
                ok = ok && __hip_atomic_load(fa.flags + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == fa.gen;
            if (__builtin_amdgcn_readfirstlane(__ballot(!ok) == 0ull)) break;
            __builtin_amdgcn_s_sleep(2);
        }
        if (i == fa.polls && lane == 0) __hip_atomic_store(fa.err, 3u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    } else if (wave == 0) {
        const uint32_t target = (fa.mode == 1 ? 1u : 8u) * (uint32_t)fa.ntrain;
        int i = 0;
        for (; i < fa.polls; ++i) {
            const uint32_t c = __hip_atomic_load(fa.sync, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (__builtin_amdgcn_readfirstlane(c) >= target) break;
            __builtin_amdgcn_s_sleep(2);
        }
        if (i == fa.polls && lane == 0) __hip_atomic_store(fa.err, 3u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        if (lane == 0 &&
            __hip_atomic_fetch_add(fa.sync + 64, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == (uint32_t)fa.nred - 1) {
            __hip_atomic_store(fa.sync, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(fa.sync + 64, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
    lds_barrier();
    if (fa.mode == 4) return;  // timing ablation (wrong results): reducers wait, then do nothing
    // slab sums: thread (half, grp, quad); half 0 sums chunks rb and rb + 2 nred, half 1 chunk rb + nred
    typedef float f4r __attribute__((ext_vector_type(4)));
    f4r(*part)[16][16] = reinterpret_cast<f4r(*)[16][16]>(smem);  // [slot][grp][quad], slot = chunk index 0..2
    const int quad = tid & 15, grp = (tid >> 4) & 15, half = tid >> 8;
    const int nmine = grp < nslabs ? (nslabs - grp + 15) / 16 : 0;
    // agent-scope loads (sc1): the slab lines other CUs stored in this launch, coherent across the XCDs' L2s
    auto ld = [&](int ch, int k) -> f4r {
        const int slab = min(grp + k * 16, nslabs - 1);
        const uint64_t w = __hip_atomic_load(
            reinterpret_cast<const uint64_t*>(slabs + (int64_t)slab * mb.n_slab + (ch * 16 + quad) * 4), __ATOMIC_RELAXED,
            __HIP_MEMORY_SCOPE_AGENT);
        const h4 v = __builtin_bit_cast(h4, w);
        return f4r{(float)v[0], (float)v[1], (float)v[2], (float)v[3]};
    };
    int chs[2] = {half ? rb + fa.nred : rb, half ? fa.nchunks : rb + 2 * fa.nred};
    int slot[2] = {half ? 1 : 0, 2};
    f4r a0[2], a1[2], v[2][8];
#pragma unroll
    for (int c = 0; c < 2; ++c) {
        a0[c] = a1[c] = f4r{0.f, 0.f, 0.f, 0.f};
        if (chs[c] >= fa.nchunks) chs[c] = -1;
#pragma unroll
        for (int u = 0; u < 8; ++u) v[c][u] = ld(chs[c] >= 0 ? chs[c] : rb, u);
    }
    for (int base = 0;;) {
#pragma unroll
        for (int c = 0; c < 2; ++c)
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const bool in = base + u < nmine;
                if (u & 1) a1[c] += in ? v[c][u] : f4r{0.f, 0.f, 0.f, 0.f};
                else a0[c] += in ? v[c][u] : f4r{0.f, 0.f, 0.f, 0.f};
            }
        base += 8;
        if (base >= nmine) break;
#pragma unroll
        for (int c = 0; c < 2; ++c)
#pragma unroll
            for (int u = 0; u < 8; ++u) v[c][u] = ld(chs[c] >= 0 ? chs[c] : rb, base + u);
    }
#pragma unroll
    for (int c = 0; c < 2; ++c)
        if (chs[c] >= 0) part[slot[c]][grp][quad] = a0[c] + a1[c];
    // the loss: reducer 0's wave 3 (the same strided per-lane sum and xor butterfly as reduce_adam_kernel)
    if (rb == 0 && wave == 3) {
        float L = 0.0f;
        for (int base = lane; base < nslabs; base += 8 * 64) {
            float lv[8];
#pragma unroll
            for (int u = 0; u < 8; ++u)
                lv[u] = __hip_atomic_load(loss_partials + min(base + 64 * u, nslabs - 1), __ATOMIC_RELAXED,
                                          __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
            for (int u = 0; u < 8; ++u) L += base + 64 * u < nslabs ? lv[u] : 0.0f;
        }
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) L += __shfl_xor(L, off, 64);
        if (lane == 0 && fa.loss_out) fa.loss_out[0] = L;
    }
    lds_barrier();
    if (pp < 0) return;
    const int lp = lane >> 2, comp = lane & 3;
    float t8[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) t8[u] = part[wave][2 * u][lp][comp] + part[wave][2 * u + 1][lp][comp];
    const float g1 = ((t8[0] + t8[1]) + (t8[2] + t8[3])) + ((t8[4] + t8[5]) + (t8[6] + t8[7]));
    adam_pack_pre(pp, g1, ain, mb, fa.oa, fa.lr_t, fa.ema_debias);
}

template <bool PADQ>
__global__ __launch_bounds__(512, 1) void train16_fused_kernel(const float* __restrict__ q, const float* __restrict__ t,
                                                               int64_t b, float n_total, float loss_scale,
                                                               const h8* __restrict__ wf, const h8* __restrict__ wb,
                                                               _Float16* __restrict__ slabs,
                                                               float* __restrict__ loss_partials, FuseArgs fa) {
    __shared__ __attribute__((aligned(16))) char smem[kLds];
    const int blk = blockIdx.x;
    if (blk >= fa.ntrain) {
        fuse_reduce(smem, blk - fa.ntrain, slabs, loss_partials, fa);
        return;
    }
    train16_split_body<16, 2, PADQ, 0>(smem, blk, q, t, b, n_total, loss_scale, wf, wb, slabs, loss_partials,
                                       HashTrainOut{});
    // count this wave (mode bit 0: this block) in once its slab / loss stores have completed (agent-scope stores)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (fa.mode == 0 || fa.mode >= 3) {
        __syncthreads();
        if (threadIdx.x == 0) __hip_atomic_store(fa.flags + blk, fa.gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else if (fa.mode == 1) {
        __syncthreads();
        if (threadIdx.x == 0) __hip_atomic_fetch_add(fa.sync, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else if ((threadIdx.x & 63) == 0) {
        __hip_atomic_fetch_add(fa.sync, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

int t16_blocks(int64_t b, int groups = 2) { return (int)((b + 64 * groups - 1) / (64 * groups)); }

}  // namespace

hipError_t launch_train16(const float* queries, const float* targets, int64_t b, float n_total, float loss_scale,
                          const _Float16* wf, const _Float16* wb, _Float16* slabs, float* loss_partials, uint64_t* stamps,
                          hipStream_t s, bool split, int groups, bool padq) {
    if (b <= 0) return hipSuccess;
    const dim3 grid(t16_blocks(b));
    const h8 *f = (const h8*)wf, *bw = (const h8*)wb;
    if (padq) {  // padded RadianceQuery records: the production shape only
        if (!split || stamps || groups != 2) return hipErrorNotSupported;
        hipLaunchKernelGGL((train16_split_kernel<16, 2, true>), grid, dim3(128 * kWaves), 0, s, queries, targets, b,
                           n_total, loss_scale, f, bw, slabs, loss_partials, HashTrainOut{});
        return hipGetLastError();
    }
    if (split && !stamps) {
        // slab stores as sc1 (AUX 16): they write through and drop the line from the XCD's L2, so the kernel does not end
        // with 5.9 MB of dirty slab lines to write back, and the reduce (on every XCD) reads them from memory either
        // way: fused step 14.2 -> 12.7 us against nt, gradients bitwise equal (profiles/r02_train/)
        if (groups == 1) {
            // 64 samples per block (debug library, A/B): twice the blocks (every CU at 16,384 samples), half the work
            // each; bitwise the decoupled-chain shape 4, but 14.5-14.7 vs 12.9-13.7 us per step
#if NRC_DEBUG_KERNELS
            hipLaunchKernelGGL((train16_split_kernel<16, 1>), dim3(t16_blocks(b, 1)), dim3(128 * kWaves), 0, s, queries,
                               targets, b, n_total, loss_scale, f, bw, slabs, loss_partials, HashTrainOut{});
            return hipGetLastError();
#else
            return hipErrorNotSupported;
#endif
        }
#if NRC_DEBUG_KERNELS
        const int tp = knob(kKnobTrainPrio);
        if (tp == 1 || tp == 2) {
            if (tp == 1)
                hipLaunchKernelGGL((train16_split_kernel<16, 2, false, 0, 1>), grid, dim3(128 * kWaves), 0, s, queries,
                                   targets, b, n_total, loss_scale, f, bw, slabs, loss_partials, HashTrainOut{});
            else
                hipLaunchKernelGGL((train16_split_kernel<16, 2, false, 0, 2>), grid, dim3(128 * kWaves), 0, s, queries,
                                   targets, b, n_total, loss_scale, f, bw, slabs, loss_partials, HashTrainOut{});
            return hipGetLastError();
        }
#endif
        hipLaunchKernelGGL((train16_split_kernel<16, 2>), grid, dim3(128 * kWaves), 0, s, queries, targets, b, n_total,
                           loss_scale, f, bw, slabs, loss_partials, HashTrainOut{});
        return hipGetLastError();
    }
#if NRC_DEBUG_KERNELS
    const dim3 block(64 * kWaves);
    if (stamps)
        hipLaunchKernelGGL((train16_kernel<true, 0>), grid, block, 0, s, queries, targets, b, n_total, loss_scale, f, bw,
                           slabs, loss_partials, stamps);
    else
        hipLaunchKernelGGL((train16_kernel<false, 0>), grid, block, 0, s, queries, targets, b, n_total, loss_scale, f, bw,
                           slabs, loss_partials, nullptr);
    return hipGetLastError();
#else
    return hipErrorNotSupported;  // the 4-wave kernel and the stamped builds live in libnrc_amd_debug.so
#endif
}

hipError_t launch_train16_fused(const float* queries, const float* targets, int64_t b, float n_total, float loss_scale,
                                const _Float16* wf, const _Float16* wb, _Float16* slabs, float* loss_partials,
                                uint32_t* sync, uint32_t* err, int polls, float* loss_out, const ModelBuffers& mb,
                                const OptimArgs& oa, hipStream_t s, bool padq, int max_blocks, int mode,
                                uint32_t gen, uint32_t* flags, int max_flags) {
    if (b <= 0 || !sync || !err || polls < 1 || mb.n_slab % 64 != 0 || mb.slab_closed != 1 || mode < 0 || mode > 4 ||
        (mode != 1 && mode != 2 && (!flags || gen == 0)))
        return hipErrorInvalidValue;
    FuseArgs fa{mb, oa, 0.0f, 0.0f, loss_out, sync, err, polls, t16_blocks(b), 0, mb.n_slab / 64, mode, gen, flags};
    if (mode != 1 && mode != 2 && fa.ntrain > max_flags) return hipErrorNotSupported;
    fa.nred = (fa.nchunks + kFuseChunksPerReducer - 1) / kFuseChunksPerReducer;
    // every block on its own CU, or the reducers would queue behind trainers and the fusion buys nothing
    if (fa.ntrain + fa.nred > max_blocks) return hipErrorNotSupported;
    adam_host_factors(oa, fa.lr_t, fa.ema_debias);
    const dim3 grid(fa.ntrain + fa.nred), block(128 * kWaves);
    const h8 *f = (const h8*)wf, *bw = (const h8*)wb;
    if (padq)
        hipLaunchKernelGGL(train16_fused_kernel<true>, grid, block, 0, s, queries, targets, b, n_total, loss_scale, f, bw,
                           slabs, loss_partials, fa);
    else
        hipLaunchKernelGGL(train16_fused_kernel<false>, grid, block, 0, s, queries, targets, b, n_total, loss_scale, f,
                           bw, slabs, loss_partials, fa);
    return hipGetLastError();
}

hipError_t launch_train16_hash(const float* queries, const float* targets, int64_t b, float n_total, float loss_scale,
                               const _Float16* wf, const _Float16* wb, _Float16* slabs, float* loss_partials,
                               const HashTrainOut& ho, hipStream_t s, bool padq, int groups) {
    if (b <= 0) return hipSuccess;
    if (!ho.table || !ho.pos || !ho.dy || ho.bcap < (int64_t)t16_blocks(b) * 128) return hipErrorInvalidValue;
    const dim3 grid(t16_blocks(b)), block(128 * kWaves);
    const h8 *f = (const h8*)wf, *bw = (const h8*)wb;
    if (groups == 1) {  // 64-sample blocks (A/B, knob t16_groups = 1): every CU at 16,384 samples, twice the slabs
        if (!ho.feat) return hipErrorNotSupported;
        const dim3 g1(t16_blocks(b, 1));
        if (padq)
            hipLaunchKernelGGL((train16_split_kernel<16, 1, true, 3>), g1, block, 0, s, queries, targets, b, n_total,
                               loss_scale, f, bw, slabs, loss_partials, ho);
        else
            hipLaunchKernelGGL((train16_split_kernel<16, 1, false, 3>), g1, block, 0, s, queries, targets, b, n_total,
                               loss_scale, f, bw, slabs, loss_partials, ho);
        return hipGetLastError();
    }
    if (ho.feat && padq)
        hipLaunchKernelGGL((train16_split_kernel<16, 2, true, 3>), grid, block, 0, s, queries, targets, b, n_total,
                           loss_scale, f, bw, slabs, loss_partials, ho);
    else if (ho.feat)
        hipLaunchKernelGGL((train16_split_kernel<16, 2, false, 3>), grid, block, 0, s, queries, targets, b, n_total,
                           loss_scale, f, bw, slabs, loss_partials, ho);
    else if (!padq)  // the gathering encoder (A/B: knob hash_infer = 1)
        hipLaunchKernelGGL((train16_split_kernel<16, 2, false, 1>), grid, block, 0, s, queries, targets, b, n_total,
                           loss_scale, f, bw, slabs, loss_partials, ho);
    else
        return hipErrorNotSupported;
    return hipGetLastError();
}

}  // namespace nrc_amd
