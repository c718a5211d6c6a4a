// Fused grid-NeRF field head on MFMA (gfx950): the sigma MLP
// 32 -> 64 -> ReLU -> 64 -> ReLU -> 4, trunc_exp density with the Gaussian
// blob, sigmoid albedo — forward, and backward with the weight gradients.
//
// Behavioural spec: nerf/network_grid.py:13-32 (MLP), :72-87 (common_forward:
// sigma = trunc_exp(h0 + 5 exp(-|x|^2 / 0.08)), albedo = sigmoid(h[1:4])),
// activation.py:5-18 (trunc_exp), run under torch.autocast(fp16)
// (nerf/utils.py train_step), i.e. f16 GEMMs with f32 accumulation and f16
// activations, f32 sigma.
//
// The reference runs this as 3 hipBLASLt GEMMs + ~15 elementwise kernels
// forward and ~25 backward, every activation round-tripping HBM.  Here one
// kernel holds a 16-sample tile in registers through all three layers:
//
//   v_mfma_f32_16x16x32_f16, operand maps (lane l, c = l & 15, h = l >> 4):
//     A[i = c][k = 8h + j], B[k = 8h + j][col = c], D[row = 4h + r][col = c]
//
// Layers are computed transposed (H^T = W X^T): the sample sits on the lane
// (column) and the neurons in the accumulator registers, so each layer's
// accumulator tile is directly the next layer's B operand — summed over its
// row index with the k order permuted (element j of lane group h is neuron
// 32s + 16(j >> 2) + 4h + (j & 3) of k-step s); the A operand (weights) is
// read from LDS in the same permuted order.  The backward recomputes the
// forward from the saved encoder features (no activations are stored), runs
// the three transposed-weight products, writes the encoder gradient directly
// in the [L, B, C] layout the sliced grid backward walks, and forms the
// weight gradients as MFMAs over 32-sample k-steps from a per-wave LDS image
// of the activations.  Per-workgroup partial sums + a fixed-order reduction
// make the weight gradients deterministic.
#include "field_common.h"

namespace dfhip {
namespace fm {

// ------------------------------------------------------------------ forward
// Grid encoding + MLP + heads in one pass: a wave takes 16 samples; lane
// group h gathers levels {h, h+4, h+8, h+12} of its sample (32 independent
// table loads in flight per lane), the features go straight into the MLP's
// B operand, and are also written (permuted order, 16 B per lane) for the
// backward.  xyz in [-bound, bound] is mapped to [0, 1] as grid.py:142 does.
template <typename E, typename rgb_t, bool QUAD>
__global__ __launch_bounds__(256, 5) void k_field_fwd_fused(
    const float *__restrict__ xyz, float bound, const E *__restrict__ table,
    const u32x4 *__restrict__ quads, const int32_t *__restrict__ offsets, ge::Levels lv, uint32_t gridtype, int align_corners,
    const float *w1, const float *b1, const float *w2, const float *b2, const float *w3,
    const float *b3, E *__restrict__ enc, float *__restrict__ sigma,
    rgb_t *__restrict__ rgb, uint32_t cap, const int32_t *__restrict__ m_dev) {
    typedef typename Elem<E>::v8 v8;
    __shared__ WeightsG<E> W;
    __shared__ LevelK LK[kLevels];
    const bool align = align_corners != 0;
    load_weights<true>(W, nullptr, w1, b1, w2, b2, w3, b3);
    stage_levels(LK, offsets, lv, gridtype, align);
    __syncthreads();
    const uint32_t M = active_count(m_dev, cap);
    const int lane = threadIdx.x & 63, c = lane & 15, h = lane >> 4;
    const uint32_t waves = gridDim.x * (blockDim.x >> 6);
    const uint32_t tiles = ceil_div(M, 16u);
    // (x + bound) / (2 bound) (grid.py:142): for a power-of-two bound the
    // quotient is the product with the exact reciprocal (no division sequence)
    const float ext = 2.0f * bound;
    const bool pow2 = (__float_as_uint(ext) & 0x007FFFFFu) == 0u && ext >= 1.17549435e-38f &&
                      ext < 1.70141183e38f;
    const float rext = 1.0f / ext;
    // positions of the wave's next tile, loaded while this one runs (12 B per
    // lane spilled at 5 waves per SIMD; still 77.5 -> 76.7 us per C2 step,
    // 415 -> 404 us textureless)
    uint32_t tile = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    float xn[3] = {0.0f, 0.0f, 0.0f};
    if (tile * 16 + c < M)
#pragma unroll
        for (int d = 0; d < 3; ++d) xn[d] = xyz[(size_t)(tile * 16 + c) * 3 + d];
    for (; tile < tiles; tile += waves) {
        // bf16: the weight operands are re-read from LDS every tile (a memory
        // clobber keeps LICM from hoisting them; hoisted, they spilled)
        if constexpr (!std::is_same<E, half_t>::value) asm volatile("" ::: "memory");
        const uint32_t sample = tile * 16 + c;
        const bool valid = sample < M;
        float x[3] = {xn[0], xn[1], xn[2]}, x01[3] = {-1.0f, -1.0f, -1.0f};
        const uint32_t nsample = (tile + waves) * 16 + c;
        if (nsample < M)
#pragma unroll
            for (int d = 0; d < 3; ++d) xn[d] = xyz[(size_t)nsample * 3 + d];
        if (valid)
#pragma unroll
            for (int d = 0; d < 3; ++d)
                x01[d] = pow2 ? (x[d] + bound) * rext : (x[d] + bound) / ext;
        const v8 xb = valid ? grid_features<E, QUAD>(table, LK, align, x01, h, quads) : v8{};
        if (enc && valid) *reinterpret_cast<v8 *>(enc + (size_t)sample * kIn + 8 * h) = xb;
        FwdG<E> F;
        forward_tile(W, xb, c, h, F);
        // lane group h holds output h: density (h = 0) or albedo channel h - 1
        if (valid) {
            if (h == 0) {
                sigma[sample] = expf((float)(E)F.o[0] + gaussian(x));
            } else {
                const float v = (float)(E)F.o[0];
                rgb[(size_t)sample * 3 + h - 1] = (rgb_t)(E)(1.0f / (1.0f + expf(-v)));
            }
        }
    }
}

template <typename rgb_t>
__global__ __launch_bounds__(256) void k_field_fwd(const half_t *__restrict__ enc,
                                                   const float *__restrict__ xyz,
                                                   const float *w1, const float *b1,
                                                   const float *w2, const float *b2,
                                                   const float *w3, const float *b3,
                                                   float *__restrict__ sigma,
                                                   rgb_t *__restrict__ rgb, uint32_t M) {
    __shared__ Weights W;
    load_weights<false>(W, nullptr, w1, b1, w2, b2, w3, b3);
    __syncthreads();
    const int lane = threadIdx.x & 63, c = lane & 15, h = lane >> 4;
    const uint32_t waves = gridDim.x * (blockDim.x >> 6);
    const uint32_t tiles = ceil_div(M, 16u);
    const uint32_t tile0 = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    half8 xb = tile0 < tiles ? load_x(enc, tile0 * 16 + c, M, h) : half8{};
    for (uint32_t tile = tile0; tile < tiles; tile += waves) {
        const uint32_t sample = tile * 16 + c;
        // prefetch the next tile's features while this one runs
        const half8 xn = tile + waves < tiles ? load_x(enc, (tile + waves) * 16 + c, M, h) : half8{};
        float x[3] = {0.0f, 0.0f, 0.0f};
        if (h == 0 && sample < M)
#pragma unroll
            for (int d = 0; d < 3; ++d) x[d] = xyz[(size_t)sample * 3 + d];
        Fwd F;
        forward_tile(W, xb, c, h, F);
        xb = xn;
        if (sample < M) {  // lane group h holds output h
            if (h == 0) {
                sigma[sample] = expf((float)(half_t)F.o[0] + gaussian(x));
            } else {
                const float v = (float)(half_t)F.o[0];
                rgb[(size_t)sample * 3 + h - 1] = (rgb_t)(half_t)(1.0f / (1.0f + expf(-v)));
            }
        }
    }
}

// The MLP alone (network_grid.py:13-32: the reference's sigma_net module, no
// heads): h [cap, 4] in E, output h of sample c on lane group h as autocast's
// f16 (bf16) linear output.  Rows [M, cap) of a capacity-sized batch (M =
// *m_dev) are written as zeros, so whatever reads the whole batch stays finite.
template <typename E>
__global__ __launch_bounds__(256) void k_mlp_fwd(const E *__restrict__ x, const float *w1,
                                                 const float *b1, const float *w2,
                                                 const float *b2, const float *w3,
                                                 const float *b3, E *__restrict__ out,
                                                 uint32_t cap, const int32_t *__restrict__ m_dev) {
    typedef typename Elem<E>::v8 v8;
    __shared__ WeightsG<E> W;
    load_weights<false>(W, nullptr, w1, b1, w2, b2, w3, b3);
    __syncthreads();
    const uint32_t M = active_count(m_dev, cap);
    const int lane = threadIdx.x & 63, c = lane & 15, h = lane >> 4;
    const uint32_t waves = gridDim.x * (blockDim.x >> 6);
    const uint32_t tiles = ceil_div(M, 16u);
    const uint32_t tile0 = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    v8 xb = tile0 < tiles ? load_x(x, tile0 * 16 + c, M, h) : v8{};
    for (uint32_t tile = tile0; tile < tiles; tile += waves) {
        const uint32_t sample = tile * 16 + c;
        const v8 xn = tile + waves < tiles ? load_x(x, (tile + waves) * 16 + c, M, h) : v8{};
        FwdG<E> F;
        forward_tile(W, xb, c, h, F);
        xb = xn;
        if (sample < M) out[(size_t)sample * kOut + h] = (E)F.o[0];
    }
    // the rows past the live count: zeros (8 bytes per row)
    typedef uint32_t u2 __attribute__((ext_vector_type(2)));
    for (size_t r = (size_t)M + (size_t)blockIdx.x * blockDim.x + threadIdx.x; r < cap;
         r += (size_t)gridDim.x * blockDim.x)
        *reinterpret_cast<u2 *>(out + r * kOut) = u2{0u, 0u};
}

// ------------------------------------------------------------------ backward
// Workgroup = 4 waves, two workgroups per CU (76 KB of LDS each), persistent
// over rounds.  Per round each wave takes one 16-sample tile: recomputes the
// forward from the saved features, runs the three transposed-weight products
// (sample on the lane, neurons in the accumulator registers), writes the
// encoder gradient in the [L, cap, C] layout the binned grid backward reads,
// and stores its activations into a [sample][neuron] LDS image of the tile —
// each lane's four neurons of one tile as ONE 8-byte write.  After a
// workgroup barrier the weight gradients of the round's 64 samples are formed
// with v_mfma_f32_16x16x16_f16, k = sample: both operands (neuron on the lane,
// four samples in the registers) come straight from the images with
// ds_read_b64_tr_b16.  The 37 output tiles (W1 8, W2 16, W3 4, and the three
// bias vectors as products with a ones operand, 9) are split over the four
// waves, so a wave holds at most 10 accumulator tiles instead of all of them:
// 2 waves per SIMD instead of 1, no per-element LDS writes, no bias VALU sums.
// Each partial entry is written by exactly one lane of the workgroup; the
// fixed-order k_field_wgrad_sum over workgroups keeps the result deterministic.
constexpr int kBwdWaves = 4;
// Weight operands held in registers for the whole kernel instead of re-read
// from LDS every tile (bit 0: W2 of the forward and W2^T, 64 VGPRs; bit 1:
// W1^T; bit 2: W3^T; bit 3: the forward's W1; bit 4: the forward's W3).
// Field backward per C2 step / textureless step: none 107 / 660 us, bit 0
// 94 / 578, bits 0-2 92 / 558, all five 90 / 545 (250 VGPRs, still 2 waves
// per SIMD).  The forward kernel's W2 in registers (4 waves per SIMD instead
// of 5) was slower: 80 -> 83 us.
#ifndef DFHIP_BWD_WREG
#define DFHIP_BWD_WREG 31
#endif
constexpr int kBwdWreg = DFHIP_BWD_WREG;
#ifndef DFHIP_BWD_PINGPONG
#define DFHIP_BWD_PINGPONG 0
#endif
constexpr int kStLd = 312;  // stage row stride (halves): 156 dwords = 4 mod 64 -> the
                            // 32 lanes of an 8-byte write hit 64 distinct banks
constexpr int kColX = 0, kColA1 = 32, kColA2 = 96, kColD1 = 160, kColD2 = 224, kColDO = 288;

template <typename E>
struct StageT {
    E v[16 * kStLd];   // [sample][x | a1 | a2 | d1 | d2 | dO(16, rows 4.. zero)]
};

typedef __fp16 fp16x4_t __attribute__((__vector_size__(4 * sizeof(__fp16))));

// Operand of v_mfma_f32_16x16x16_{f16,bf16} with the neuron on the lane: lane
// (g = l >> 4, i = l & 15) gets columns c0 + i of sample rows 4g .. 4g + 3
// (ds_read_b64_tr_b16: lane 4q + p of the group supplies row 4g + q, columns
// c0 + 4p .. c0 + 4p + 3).
template <typename E>
__device__ __forceinline__ typename Elem<E>::v4 tr_operand(const StageT<E> &S, int c0, int lane) {
    const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
    const E *src = S.v + (4 * g + q) * kStLd + c0 + 4 * p;
    typename Elem<E>::v4 out;
    if constexpr (std::is_same<E, half_t>::value) {
        const fp16x4_t r = __builtin_amdgcn_ds_read_tr16_b64_v4f16(
            (__attribute__((address_space(3))) fp16x4_t *)src);
        __builtin_memcpy(&out, &r, sizeof(out));
    } else {
        out = __builtin_amdgcn_ds_read_tr16_b64_v4bf16(
            (__attribute__((address_space(3))) bf4 *)src);
    }
    return out;
}

__device__ __forceinline__ f4 mfma16(half4 a, half4 b, f4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x16f16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ f4 mfma16(bf4 a, bf4 b, f4 c) {
    typedef short s4 __attribute__((ext_vector_type(4)));
    s4 x, y;
    __builtin_memcpy(&x, &a, sizeof(x));
    __builtin_memcpy(&y, &b, sizeof(y));
    return __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(x, y, c, 0, 0, 0);
}

template <typename E>
__device__ __forceinline__ void st_write4(StageT<E> &S, int sample, int col, E v0, E v1, E v2,
                                          E v3) {
    *reinterpret_cast<typename Elem<E>::v4 *>(S.v + sample * kStLd + col) =
        typename Elem<E>::v4{v0, v1, v2, v3};
}

// One wave's inputs for a 16-sample tile: encoder features (every lane), and
// the incoming gradient of the lane group's output (h = 0: the density's, with
// the position for the Gaussian blob; h > 0: albedo channel h - 1's) — as
// loaded (no conversion), so a prefetch does not wait for its loads.
template <typename E, typename rgb_t>
struct TileIn {
    typename Elem<E>::v8 xb;
    float xyz[3], gs;
    rgb_t grgb;
};

// MLP_ONLY (the plain MLP, k_mlp_fwd's backward): grad_rgb is dh [M, 4] and
// lane group h takes output h's gradient.
template <typename E, typename rgb_t, bool MLP_ONLY = false>
__device__ __forceinline__ void load_tile(TileIn<E, rgb_t> &g, uint32_t tile, const E *enc,
                                          const float *xyz, const float *grad_sigma,
                                          const rgb_t *grad_rgb, uint32_t M, int c, int h) {
    const uint32_t sample = tile * 16 + c;
    g.xb = load_x(enc, sample, M, h);
    if constexpr (MLP_ONLY) {
        g.gs = 0.0f;
        g.xyz[0] = g.xyz[1] = g.xyz[2] = 0.0f;
        g.grgb = sample < M ? grad_rgb[(size_t)sample * kOut + h] : (rgb_t)0.0f;
        return;
    }
    const bool v = (h == 0) && sample < M;
#pragma unroll
    for (int d = 0; d < 3; ++d) g.xyz[d] = v ? xyz[(size_t)sample * 3 + d] : 0.0f;
    g.gs = v ? grad_sigma[sample] : 0.0f;
    g.grgb = (h > 0 && sample < M) ? grad_rgb[(size_t)sample * 3 + h - 1] : (rgb_t)0.0f;
}

// PERM: enc holds the fused forward's permuted feature order (k_field_fwd_fused);
// otherwise the natural [M, 32] encoder output.  M = *m_dev (clamped to cap)
// when m_dev is given; d_enc is [16, cap, 2].  MLP_ONLY: the plain MLP's
// backward (k_mlp_fwd): grad_rgb is dh [cap, 4] in E, no heads, and d_enc is
// the natural [cap, 32] feature gradient (rows [M, cap) written as zeros).
template <typename E, typename rgb_t, bool PERM, bool MLP_ONLY = false>
__global__ __launch_bounds__(64 * kBwdWaves, 2) void k_field_bwd(
    const E *__restrict__ enc, const float *__restrict__ xyz, const float *w1,
    const float *b1, const float *w2, const float *b2, const float *w3, const float *b3,
    const float *__restrict__ grad_sigma, const rgb_t *__restrict__ grad_rgb, uint32_t cap,
    const int32_t *__restrict__ m_dev,
    E *__restrict__ d_enc,          // [16, cap, 2] (level-major)
    float *__restrict__ partial) {  // [gridDim.x, kParams]
    typedef typename Elem<E>::v8 v8;
    typedef typename Elem<E>::v4 v4;
    __shared__ WeightsG<E> W;
    __shared__ WeightsTG<E> T;
    __shared__ StageT<E> stage[kBwdWaves];
    load_weights<PERM>(W, &T, w1, b1, w2, b2, w3, b3);
    const uint32_t M = active_count(m_dev, cap);
    const int wave = threadIdx.x >> 6;
    const int lane = threadIdx.x & 63, c = lane & 15, h = lane >> 4;
    StageT<E> &S = stage[wave];
    __syncthreads();

    // this wave's accumulator tiles (see the ownership table below)
    f4 acc[10];
#pragma unroll
    for (int i = 0; i < 10; ++i) acc[i] = f4{0, 0, 0, 0};
    const v4 ones = v4{(E)1.0f, (E)1.0f, (E)1.0f, (E)1.0f};
    // weight operands kept in registers (kBwdWreg)
    v8 w2op[4][2], w2top[4][2], w1top[2][2], w3top[4], w1op[4], w3op[2];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) {
            if (kBwdWreg & 1) {
                w2op[u][s2] = a_perm(W.w2, kLd64, 16 * u + c, s2, h);
                w2top[u][s2] = a_perm(T.w2t, kLd64, 16 * u + c, s2, h);
            }
            if ((kBwdWreg & 2) && u < 2) w1top[u][s2] = a_perm(T.w1t, kLd64, 16 * u + c, s2, h);
        }
        if (kBwdWreg & 4) w3top[u] = a_nat(T.w3t, kLd32, 16 * u + c, 0, h);
        if (kBwdWreg & 8) w1op[u] = a_nat(W.w1, kLd32, 16 * u + c, 0, h);
        if ((kBwdWreg & 16) && u < 2) w3op[u] = a_perm(W.w3, kLd64, c, u, h);
    }

    const uint32_t tiles = ceil_div(M, 16u);
    const uint32_t per_round = gridDim.x * kBwdWaves;
    const uint32_t rounds = ceil_div(tiles, per_round);
    // dO^T image columns 4..15 are zero for good (each round writes 0..3)
    st_write4(S, c, kColDO + 4 * h, (E)0.0f, (E)0.0f, (E)0.0f, (E)0.0f);
    // one round: the tile's forward recompute, backward and its share of the
    // weight gradients (every wave runs the same number of rounds: barriers)
    auto round_of = [&](const TileIn<E, rgb_t> &cur, uint32_t tile) {
        const uint32_t sample = tile * 16 + c;
        const bool valid = sample < M;
        FwdG<E, true> F;  // packed activations (f16 pairs per VGPR)
        forward_tile<E, true, (kBwdWreg & 1) != 0, (kBwdWreg & 8) != 0, (kBwdWreg & 16) != 0>(
            W, cur.xb, c, h, F, w2op, w1op, w3op);
        // dL/d(output h), in E as autocast's backward produces it: lane group h
        // holds output h (F.o[0]) and its incoming gradient
        E dOh = (E)0.0f;
        if (MLP_ONLY) {
            dOh = valid ? (E)cur.grgb : (E)0.0f;
        } else if (valid) {
            if (h == 0) {
                const float y = (float)(E)F.o[0] + gaussian(cur.xyz);
                // trunc_exp backward (activation.py:14-18): g * exp(clamp(y, -15, 15))
                const float yc = fminf(fmaxf(y, -15.0f), 15.0f);
                dOh = (E)(cur.gs * expf(yc));
            } else {
                const float a = (float)(E)(1.0f / (1.0f + expf(-(float)(E)F.o[0])));
                const float g = (float)(E)(float)cur.grgb;
                dOh = (E)(g * (1.0f - a) * a);  // sigmoid_backward in E (opmath f32)
            }
        }
        // B operand of W3^T dO^T: output h at k = 8 h (T.w3t's layout)
        const v8 dob = v8{dOh, (E)0.0f, (E)0.0f, (E)0.0f, (E)0.0f, (E)0.0f, (E)0.0f, (E)0.0f};
        // ReLU mask of an accumulator tile by the layer's activations
        constexpr bool kBf = std::is_same<E, bf16_t>::value;
        auto mask = [&](const auto &act, const f4 &d, auto &dst) {
            if constexpr (kBf) {
                const f4 m = {(float)act[0] > 0.0f ? d[0] : 0.0f,
                              (float)act[1] > 0.0f ? d[1] : 0.0f,
                              (float)act[2] > 0.0f ? d[2] : 0.0f,
                              (float)act[3] > 0.0f ? d[3] : 0.0f};
                dst = __builtin_convertvector(m, bf4);
            } else {
                // f16 ReLU backward on packed pairs: act is a ReLU output (+-0
                // or positive), so act > 0 <=> its magnitude bits are nonzero;
                // ((x & 0x7fff) + 0x7fff) sets bit 15 exactly then, and
                // (bit >> 15) * 0xffff widens it to the half's mask
                typedef uint32_t u2 __attribute__((ext_vector_type(2)));
                const half4 dh = __builtin_convertvector(d, half4);
                u2 ab, db;
                __builtin_memcpy(&ab, &act, 8);
                __builtin_memcpy(&db, &dh, 8);
                const u2 nz = ((ab & 0x7FFF7FFFu) + 0x7FFF7FFFu) & 0x80008000u;
                const u2 r = db & ((nz >> 15u) * 0xFFFFu);
                __builtin_memcpy(&dst, &r, 8);
            }
        };
        // hidden layer 2: dA2^T = W3^T dO^T, ReLU mask
        typename TilesT<E, true>::type dz2;
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const f4 d = mfma((kBwdWreg & 4) ? w3top[u] : a_nat(T.w3t, kLd32, 16 * u + c, 0, h),
                              dob, f4{0, 0, 0, 0});
            mask(F.a2[u], d, dz2[u]);
        }
        // hidden layer 1: dA1^T = W2^T dZ2^T, ReLU mask
        typename TilesT<E, true>::type dz1;
#pragma unroll
        for (int t = 0; t < 4; ++t) {
            f4 d = f4{0, 0, 0, 0};
#pragma unroll
            for (int s2 = 0; s2 < 2; ++s2)
                d = mfma((kBwdWreg & 1) ? w2top[t][s2] : a_perm(T.w2t, kLd64, 16 * t + c, s2, h),
                         b_from_tiles(dz2, s2), d);
            mask(F.a1[t], d, dz1[t]);
        }
        // encoder features: dX^T = W1^T dZ1^T -> [L, B, C] directly
#pragma unroll
        for (int f = 0; f < 2; ++f) {
            f4 d = f4{0, 0, 0, 0};
#pragma unroll
            for (int s2 = 0; s2 < 2; ++s2)
                d = mfma((kBwdWreg & 2) ? w1top[f][s2] : a_perm(T.w1t, kLd64, 16 * f + c, s2, h),
                         b_from_tiles(dz1, s2), d);
            if (MLP_ONLY && valid) {
                // natural [cap, 32]: features 16f + 4h .. 16f + 4h + 3 of the sample
                *reinterpret_cast<v4 *>(d_enc + (size_t)sample * kIn + 16 * f + 4 * h) =
                    v4{(E)d[0], (E)d[1], (E)d[2], (E)d[3]};
            } else if (valid) {
                // features 16f + 4h + r = level 8f + 2h + (r >> 1), channel r & 1
                const uint32_t lv = 8 * f + 2 * h;
                typedef E e2v __attribute__((ext_vector_type(2)));
                *reinterpret_cast<e2v *>(d_enc + ((size_t)lv * cap + sample) * 2) =
                    e2v{(E)d[0], (E)d[1]};
                *reinterpret_cast<e2v *>(d_enc + ((size_t)(lv + 1) * cap + sample) * 2) =
                    e2v{(E)d[2], (E)d[3]};
            }
        }
        // [sample][neuron] image of the tile (invalid samples: dO = 0 so every
        // gradient row is zero and they add nothing below)
        *reinterpret_cast<v8 *>(S.v + c * kStLd + kColX + 8 * h) = cur.xb;
#pragma unroll
        for (int t = 0; t < 4; ++t) {
            const int col = 16 * t + 4 * h;
            *reinterpret_cast<v4 *>(S.v + c * kStLd + kColA1 + col) = F.a1[t];
            *reinterpret_cast<v4 *>(S.v + c * kStLd + kColA2 + col) = F.a2[t];
            *reinterpret_cast<v4 *>(S.v + c * kStLd + kColD1 + col) = dz1[t];
            *reinterpret_cast<v4 *>(S.v + c * kStLd + kColD2 + col) = dz2[t];
        }
        S.v[c * kStLd + kColDO + h] = dOh;  // columns 4..15 stay zero
        __syncthreads();
        // weight gradients over the round's 4 x 16 samples.  Tile ownership:
        //   wave 0 / 1: W2 rows tn in {0,1} / {2,3} x 4 column tiles, b2 rows tn
        //   wave 2 / 3: W1 rows tn in {0,1} / {2,3} x 2 feature tiles, b1 rows tn,
        //               W3 columns tm in {0,1} / {2,3}; wave 2 also b3
        // k = 32 samples per MFMA (v_mfma_f32_16x16x32, the full-rate form on
        // gfx950): operand element jj of lane group g is sample row 4g + (jj & 3)
        // of stage st + (jj >> 2) — two transposed reads, the same map for both
        // operands
        auto tr2 = [&](int st, int c0) {
            const v4 lo = tr_operand(stage[st], c0, lane);
            const v4 hi = tr_operand(stage[st + 1], c0, lane);
            return (v8)__builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
        };
        const v8 ones8 = __builtin_shufflevector(ones, ones, 0, 1, 2, 3, 4, 5, 6, 7);
#pragma unroll
        for (int st = 0; st < kBwdWaves; st += 2) {
            if (wave < 2) {
#pragma unroll
                for (int k = 0; k < 2; ++k) {
                    const int tn = 2 * wave + k;
                    const v8 a = tr2(st, kColD2 + 16 * tn);
#pragma unroll
                    for (int tm = 0; tm < 4; ++tm)
                        acc[5 * k + tm] = mfma(a, tr2(st, kColA1 + 16 * tm), acc[5 * k + tm]);
                    acc[5 * k + 4] = mfma(a, ones8, acc[5 * k + 4]);
                }
            } else {
                const int w2i = wave - 2;
#pragma unroll
                for (int k = 0; k < 2; ++k) {
                    const int tn = 2 * w2i + k;
                    const v8 a = tr2(st, kColD1 + 16 * tn);
#pragma unroll
                    for (int tf = 0; tf < 2; ++tf)
                        acc[3 * k + tf] = mfma(a, tr2(st, kColX + 16 * tf), acc[3 * k + tf]);
                    acc[3 * k + 2] = mfma(a, ones8, acc[3 * k + 2]);
                }
                const v8 ao = tr2(st, kColDO);
#pragma unroll
                for (int k = 0; k < 2; ++k)
                    acc[6 + k] = mfma(ao, tr2(st, kColA2 + 16 * (2 * w2i + k)), acc[6 + k]);
                if (wave == 2) acc[8] = mfma(ao, ones8, acc[8]);
            }
        }
        __syncthreads();  // the images are rewritten next round
    };
    // two input buffers in turn: round r + 1's loads are issued before round
    // r runs and first waited on in round r + 1 (a copy of the prefetched
    // registers at the end of each round would wait for them there)
    uint32_t tile = blockIdx.x * kBwdWaves + wave;
#if DFHIP_BWD_PINGPONG
    TileIn<E, rgb_t> ta, tb;
    load_tile<E, rgb_t>(ta, tile, enc, xyz, grad_sigma, grad_rgb, M, c, h);
    for (uint32_t round = 0; round < rounds; round += 2) {
        load_tile<E, rgb_t>(tb, tile + per_round, enc, xyz, grad_sigma, grad_rgb, M, c, h);
        round_of(ta, tile);
        tile += per_round;
        if (round + 1 >= rounds) break;  // uniform
        load_tile<E, rgb_t>(ta, tile + per_round, enc, xyz, grad_sigma, grad_rgb, M, c, h);
        round_of(tb, tile);
        tile += per_round;
    }
#else
    TileIn<E, rgb_t> cur;
    load_tile<E, rgb_t, MLP_ONLY>(cur, tile, enc, xyz, grad_sigma, grad_rgb, M, c, h);
    for (uint32_t round = 0; round < rounds; ++round, tile += per_round) {
        TileIn<E, rgb_t> nxt;  // the next round's inputs, loaded while this one runs
        load_tile<E, rgb_t, MLP_ONLY>(nxt, tile + per_round, enc, xyz, grad_sigma, grad_rgb, M, c,
                                      h);
        round_of(cur, tile);
        cur = nxt;
    }
#endif
    if constexpr (MLP_ONLY) {
        // feature-gradient rows past the live count: zeros (64 bytes per row)
        for (size_t i = (size_t)M * 4 + (size_t)blockIdx.x * blockDim.x + threadIdx.x;
             i < (size_t)cap * 4; i += (size_t)gridDim.x * blockDim.x)
            reinterpret_cast<u32x4 *>(d_enc)[i] = u32x4{0u, 0u, 0u, 0u};
    }

    // ---- this workgroup's partial: every entry written by exactly one lane.
    // Accumulator element r of lane (c, h): row 4h + r, column c of the tile.
    float *out = partial + (size_t)blockIdx.x * kParams;
    if (wave < 2) {
#pragma unroll
        for (int k = 0; k < 2; ++k) {
            const int tn = 2 * wave + k;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int n = 16 * tn + 4 * h + r;
#pragma unroll
                for (int tm = 0; tm < 4; ++tm)
                    out[kOffW2 + n * kHid + 16 * tm + c] = acc[5 * k + tm][r];
                if (c == 0) out[kOffB2 + n] = acc[5 * k + 4][r];
            }
        }
    } else {
        const int w2i = wave - 2;
#pragma unroll
        for (int k = 0; k < 2; ++k) {
            const int tn = 2 * w2i + k;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int n = 16 * tn + 4 * h + r;
#pragma unroll
                for (int tf = 0; tf < 2; ++tf) {
                    const int p = 16 * tf + c;  // layer-1 input position
                    out[kOffW1 + n * kIn + (PERM ? perm_feature(p) : p)] = acc[3 * k + tf][r];
                }
                if (c == 0) out[kOffB1 + n] = acc[3 * k + 2][r];
            }
            if (h == 0)
#pragma unroll
                for (int r = 0; r < 4; ++r)
                    out[kOffW3 + r * kHid + 16 * (2 * w2i + k) + c] = acc[6 + k][r];
        }
        if (wave == 2 && lane == 0)
#pragma unroll
            for (int r = 0; r < 4; ++r) out[kOffB3 + r] = acc[8][r];
    }
}

// Sum the per-workgroup partials (fixed order) into the six f32 gradients:
// a block takes 64 parameters; its 16 part-lanes sum the parts p = j, j+16,
// ... of each, then lane j = 0 adds the 16 lane sums in order.
__global__ __launch_bounds__(1024) void k_field_wgrad_sum(const float *__restrict__ partial,
                                                          uint32_t parts, float *gw1, float *gb1,
                                                          float *gw2, float *gb2, float *gw3,
                                                          float *gb3, int accumulate) {
    __shared__ float lane_sum[16][64];
    const int col = threadIdx.x & 63, j = threadIdx.x >> 6;
    const int i = blockIdx.x * 64 + col;
    float s = 0.0f;
    if (i < kParams) {
        // parts j, j + 16, ... added in that order; eight loads in flight
        uint32_t p = j;
        for (; p + 7 * 16 < parts; p += 8 * 16) {
            float x[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) x[u] = partial[(size_t)(p + 16 * u) * kParams + i];
#pragma unroll
            for (int u = 0; u < 8; ++u) s += x[u];
        }
        for (; p < parts; p += 16) s += partial[(size_t)p * kParams + i];
    }
    lane_sum[j][col] = s;
    __syncthreads();
    if (j != 0 || i >= kParams) return;
    s = 0.0f;
#pragma unroll
    for (int q = 0; q < 16; ++q) s += lane_sum[q][col];
    float *dst;
    int k;
    if (i < kOffB1) { dst = gw1; k = i - kOffW1; }
    else if (i < kOffW2) { dst = gb1; k = i - kOffB1; }
    else if (i < kOffB2) { dst = gw2; k = i - kOffW2; }
    else if (i < kOffW3) { dst = gb2; k = i - kOffB2; }
    else if (i < kOffB3) { dst = gw3; k = i - kOffW3; }
    else { dst = gb3; k = i - kOffB3; }
    dst[k] = accumulate ? dst[k] + s : s;
}

static uint32_t bwd_blocks(uint32_t M) {
    const uint32_t cus = device_cus();
    const uint32_t want = ceil_div(ceil_div(M, 16u), (uint32_t)kBwdWaves);
    const uint32_t cap = 2u * cus;  // two workgroups per CU
    return want < cap ? (want ? want : 1u) : cap;
}
// partial rows the backward writes for M rows (k_field_wgrad_sum's parts)
static uint32_t bwd_parts(uint32_t M) { return bwd_blocks(M); }

}  // namespace fm
}  // namespace dfhip

using namespace dfhip;
using namespace dfhip::fm;

extern "C" uint32_t dfhip_field_mlp_params(void) { return (uint32_t)kParams; }

extern "C" uint32_t dfhip_field_mlp_backward_parts(uint32_t M) { return bwd_parts(M); }

extern "C" int dfhip_field_mlp_forward(const void *enc, const float *xyz, const float *w1,
                                       const float *b1, const float *w2, const float *b2,
                                       const float *w3, const float *b3, float *sigma,
                                       void *rgb, int rgb_dtype, uint32_t M,
                                       dfhip_stream_t stream) {
    const char *name = "field_mlp_forward";
    if (M == 0) return DFHIP_OK;
    if (!enc || !xyz || !w1 || !b1 || !w2 || !b2 || !w3 || !b3 || !sigma || !rgb) {
        set_error("%s: null pointer", name);
        return DFHIP_EINVAL;
    }
    hipStream_t s = as_stream(stream);
    const uint32_t tiles = ceil_div(M, 16u);
    const uint32_t blocks = ceil_div(tiles, 4u) < 2048u ? ceil_div(tiles, 4u) : 2048u;
    if (rgb_dtype == DFHIP_F32)
        k_field_fwd<float><<<blocks, 256, 0, s>>>((const half_t *)enc, xyz, w1, b1, w2, b2, w3,
                                                  b3, sigma, (float *)rgb, M);
    else if (rgb_dtype == DFHIP_F16)
        k_field_fwd<half_t><<<blocks, 256, 0, s>>>((const half_t *)enc, xyz, w1, b1, w2, b2, w3,
                                                   b3, sigma, (half_t *)rgb, M);
    else {
        set_error("%s: rgb dtype must be f32 or f16", name);
        return DFHIP_EDTYPE;
    }
    return check_launch(name);
}

extern "C" int dfhip_field_mlp_backward(const void *enc, const float *xyz, const float *w1,
                                        const float *b1, const float *w2, const float *b2,
                                        const float *w3, const float *b3, const float *grad_sigma,
                                        const void *grad_rgb, int grad_rgb_dtype, uint32_t M,
                                        void *d_enc_lbc, float *partial, uint32_t parts,
                                        float *gw1, float *gb1, float *gw2, float *gb2,
                                        float *gw3, float *gb3, int accumulate,
                                        dfhip_stream_t stream) {
    const char *name = "field_mlp_backward";
    if (!w1 || !b1 || !w2 || !b2 || !w3 || !b3 || !gw1 || !gb1 || !gw2 || !gb2 || !gw3 || !gb3 ||
        !partial) {
        set_error("%s: null pointer", name);
        return DFHIP_EINVAL;
    }
    hipStream_t s = as_stream(stream);
    if (M > 0) {
        if (!enc || !xyz || !grad_sigma || !grad_rgb || !d_enc_lbc) {
            set_error("%s: null pointer", name);
            return DFHIP_EINVAL;
        }
        if (parts != bwd_parts(M)) {
            set_error("%s: parts must be dfhip_field_mlp_backward_parts(M) = %u (got %u)", name,
                      bwd_parts(M), parts);
            return DFHIP_EINVAL;
        }
        const uint32_t nblk = bwd_blocks(M);
#define DFHIP_BWDN(R)                                                                          \
    k_field_bwd<half_t, R, false><<<nblk, 256, 0, s>>>(                                        \
        (const half_t *)enc, xyz, w1, b1, w2, b2, w3, b3, grad_sigma, (const R *)grad_rgb, M,  \
        nullptr, (half_t *)d_enc_lbc, partial)
        if (grad_rgb_dtype == DFHIP_F32)
            DFHIP_BWDN(float);
        else if (grad_rgb_dtype == DFHIP_F16)
            DFHIP_BWDN(half_t);
#undef DFHIP_BWDN
        else {
            set_error("%s: grad_rgb dtype must be f32 or f16", name);
            return DFHIP_EDTYPE;
        }
    } else {
        parts = 1;
        (void)hipMemsetAsync(partial, 0, kParams * sizeof(float), s);
    }
    k_field_wgrad_sum<<<ceil_div((uint32_t)kParams, 64u), 1024, 0, s>>>(
        partial, parts, gw1, gb1, gw2, gb2, gw3, gb3, accumulate);
    return check_launch(name);
}

template <typename E>
static int mlp_launch(const char *name, const void *x, const float *w1, const float *b1,
                      const float *w2, const float *b2, const float *w3, const float *b3, void *h,
                      uint32_t cap, const int32_t *m_dev, hipStream_t s) {
    const uint32_t tiles = ceil_div(cap, 16u);
    const uint32_t blocks = ceil_div(tiles, 4u) < 2048u ? ceil_div(tiles, 4u) : 2048u;
    k_mlp_fwd<E><<<blocks, 256, 0, s>>>((const E *)x, w1, b1, w2, b2, w3, b3, (E *)h, cap, m_dev);
    return check_launch(name);
}

extern "C" int dfhip_mlp_forward(int elem, const void *x, const float *w1, const float *b1,
                                 const float *w2, const float *b2, const float *w3,
                                 const float *b3, void *h, uint32_t cap, const int32_t *m_dev,
                                 dfhip_stream_t stream) {
    const char *name = "mlp_forward";
    if (cap == 0) return DFHIP_OK;
    if (!x || !w1 || !b1 || !w2 || !b2 || !w3 || !b3 || !h) {
        set_error("%s: null pointer", name);
        return DFHIP_EINVAL;
    }
    if (elem == DFHIP_F16)
        return mlp_launch<half_t>(name, x, w1, b1, w2, b2, w3, b3, h, cap, m_dev,
                                  as_stream(stream));
    if (elem == DFHIP_BF16)
        return mlp_launch<bf16_t>(name, x, w1, b1, w2, b2, w3, b3, h, cap, m_dev,
                                  as_stream(stream));
    set_error("%s: elem must be f16 or bf16", name);
    return DFHIP_EDTYPE;
}

extern "C" int dfhip_mlp_backward(int elem, const void *x, const float *w1, const float *b1,
                                  const float *w2, const float *b2, const float *w3,
                                  const float *b3, const void *dh, uint32_t cap,
                                  const int32_t *m_dev, void *dx, float *partial, uint32_t parts,
                                  float *gw1, float *gb1, float *gw2, float *gb2, float *gw3,
                                  float *gb3, int accumulate, dfhip_stream_t stream) {
    const char *name = "mlp_backward";
    if (!w1 || !b1 || !w2 || !b2 || !w3 || !b3 || !gw1 || !gb1 || !gw2 || !gb2 || !gw3 || !gb3 ||
        !partial) {
        set_error("%s: null pointer", name);
        return DFHIP_EINVAL;
    }
    if (elem != DFHIP_F16 && elem != DFHIP_BF16) {
        set_error("%s: elem must be f16 or bf16", name);
        return DFHIP_EDTYPE;
    }
    hipStream_t s = as_stream(stream);
    if (cap > 0) {
        if (!x || !dh || !dx) {
            set_error("%s: null pointer", name);
            return DFHIP_EINVAL;
        }
        if (parts != bwd_parts(cap)) {
            set_error("%s: parts must be dfhip_field_mlp_backward_parts(cap) = %u (got %u)", name,
                      bwd_parts(cap), parts);
            return DFHIP_EINVAL;
        }
        const uint32_t nblk = bwd_blocks(cap);
        if (elem == DFHIP_F16)
            k_field_bwd<half_t, half_t, false, true><<<nblk, 256, 0, s>>>(
                (const half_t *)x, nullptr, w1, b1, w2, b2, w3, b3, nullptr, (const half_t *)dh,
                cap, m_dev, (half_t *)dx, partial);
        else
            k_field_bwd<bf16_t, bf16_t, false, true><<<nblk, 256, 0, s>>>(
                (const bf16_t *)x, nullptr, w1, b1, w2, b2, w3, b3, nullptr, (const bf16_t *)dh,
                cap, m_dev, (bf16_t *)dx, partial);
    } else {
        parts = 1;
        (void)hipMemsetAsync(partial, 0, kParams * sizeof(float), s);
    }
    k_field_wgrad_sum<<<ceil_div((uint32_t)kParams, 64u), 1024, 0, s>>>(
        partial, parts, gw1, gb1, gw2, gb2, gw3, gb3, accumulate);
    return check_launch(name);
}

// ------------------------------------------------------------------ grid encoding
// GridEncoder's forward for the reference's grid shape (16 levels x 2
// channels, D = 3, f16 table; gridencoder.cu:75-178) on the fused field's
// gather: a wave takes 16 samples, lane group h gathers levels h, h + 4,
// h + 8, h + 12 of its sample with the paired-corner loads (50 gathers per
// sample instead of k_grid_fwd's 128 scalar ones, every level chain of a lane
// independent), and the features are stored in the natural [B, 32] order —
// the same half arithmetic, so the same bits.  Rows [M, B) of a
// capacity-sized batch (M = *m_dev) are written as zeros; bound > 0: raw
// positions mapped as grid.py:142.
__global__ __launch_bounds__(256) void k_grid_fwd_tiles(const float *__restrict__ inputs,
                                                       float bound, const half_t *__restrict__ table,
                                                       const int32_t *__restrict__ offsets,
                                                       ge::Levels lv, uint32_t gridtype,
                                                       int align_corners,
                                                       half_t *__restrict__ out, uint32_t B,
                                                       const int32_t *__restrict__ m_dev) {
    __shared__ LevelK LK[kLevels];
    stage_levels(LK, offsets, lv, gridtype, align_corners != 0);
    __syncthreads();
    const uint32_t M = active_count(m_dev, B);
    const int lane = threadIdx.x & 63, c = lane & 15, h = lane >> 4;
    const uint32_t waves = gridDim.x * (blockDim.x >> 6);
    const uint32_t tiles = ceil_div(B, 16u);
    const float ext = 2.0f * bound;
    for (uint32_t tile = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); tile < tiles;
         tile += waves) {
        const uint32_t sample = tile * 16 + c;
        if (sample >= B) continue;
        half8 f{};
        if (sample < M) {
            float x[3];
#pragma unroll
            for (int d = 0; d < 3; ++d) {
                const float v = inputs[(size_t)sample * 3 + d];
                x[d] = bound > 0.0f ? (v + bound) / ext : v;
            }
            f = grid_features<half_t>(table, LK, align_corners != 0, x, h);
        }
        // level 4 q + h, channel ch -> column 2 (4 q + h) + ch
        uint32_t *row = reinterpret_cast<uint32_t *>(out + (size_t)sample * 32);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            half2v v = half2v{f[2 * q], f[2 * q + 1]};
            uint32_t w;
            __builtin_memcpy(&w, &v, 4);
            row[4 * q + h] = w;
        }
    }
}

namespace dfhip {
// GridEncoder forward on the tile gather (k_grid_fwd_tiles) for the shapes it
// takes (gridencoder.hip dispatches here): D = 3, C = 2, L = 16, f16 table,
// no dy_dx, [B, L C] output.  Returns false when it does not apply.
bool grid_forward_tiles_f16(const float *inputs, float bound, const void *table,
                            const int32_t *offsets, uint32_t L, float S, uint32_t H,
                            uint32_t gridtype, int align_corners, void *outputs, uint32_t B,
                            const int32_t *m_dev, hipStream_t s) {
    if (L != (uint32_t)kLevels || B == 0) return false;
    const ge::Levels lv = ge::make_levels(L, S, H);
    const uint32_t tiles = ceil_div(B, 16u);
    const uint32_t want = ceil_div(tiles, 4u);
    const uint32_t blocks = want < 8192u ? want : 8192u;
    k_grid_fwd_tiles<<<blocks, 256, 0, s>>>(inputs, bound, (const half_t *)table, offsets, lv,
                                            gridtype, align_corners, (half_t *)outputs, B, m_dev);
    return true;
}
}  // namespace dfhip

// ------------------------------------------------------------------ fused grid field
static bool check_field_grid(const char *name, uint32_t L) {
    if (L != 16) {
        set_error("%s: the fused field supports the reference's 16-level x 2-channel 3-D grid "
                  "(got L=%u)", name, L);
        return false;
    }
    return true;
}

template <typename E, typename rgb_t, bool QUAD>
static void launch_field_fwd(hipStream_t s, const float *xyz, float bound, const void *table,
                             const void *quads, const int32_t *offsets, const ge::Levels &lv, uint32_t gridtype,
                             int align_corners, const float *w1, const float *b1, const float *w2,
                             const float *b2, const float *w3, const float *b3, void *enc,
                             float *sigma, void *rgb, uint32_t cap, const int32_t *m_dev) {
    // persistent waves: exactly one resident wave per slot of the chip (each
    // walks ~M / (16 * waves) tiles); more blocks than fit leave a partial
    // last round of blocks (4096 blocks at 5 waves/SIMD were 3.2 rounds)
    const uint32_t tiles = ceil_div(cap, 16u);
    const uint32_t fit = resident_blocks((const void *)k_field_fwd_fused<E, rgb_t, QUAD>, 256, 4);
    const uint32_t blocks = ceil_div(tiles, 4u) < fit ? ceil_div(tiles, 4u) : fit;
    k_field_fwd_fused<E, rgb_t, QUAD><<<blocks, 256, 0, s>>>(
        xyz, bound, (const E *)table, (const u32x4 *)quads, offsets, lv, gridtype, align_corners, w1, b1, w2, b2, w3,
        b3, (E *)enc, sigma, (rgb_t *)rgb, cap, m_dev);
}

// elem: DFHIP_F16 (table, features, activations in f16: the reference's fp16
// autocast) or DFHIP_BF16 (all of them bf16: bf16 autocast, the C5 option).
static int grid_field_forward(const char *name, int elem, const float *xyz, float bound,
                              const void *table, const void *quads, const int32_t *offsets, uint32_t L, float S,
                              uint32_t H, uint32_t gridtype, int align_corners, const float *w1,
                              const float *b1, const float *w2, const float *b2, const float *w3,
                              const float *b3, void *enc, float *sigma, void *rgb, int rgb_dtype,
                              uint32_t cap, const int32_t *m_dev, dfhip_stream_t stream) {
    if (!check_field_grid(name, L)) return DFHIP_EINVAL;
    if (!(bound > 0.0f)) {
        set_error("%s: bound must be > 0", name);
        return DFHIP_EINVAL;
    }
    if (cap == 0) return DFHIP_OK;
    if (!xyz || !table || !offsets || !w1 || !b1 || !w2 || !b2 || !w3 || !b3 || !sigma || !rgb) {
        set_error("%s: null pointer", name);
        return DFHIP_EINVAL;
    }
    hipStream_t s = as_stream(stream);
    const ge::Levels lv = ge::make_levels(L, S, H);
#define DFHIP_FWD(E, R)                                                                       \
    (quads ? launch_field_fwd<E, R, true>(s, xyz, bound, table, quads, offsets, lv, gridtype,    \
                                          align_corners, w1, b1, w2, b2, w3, b3, enc, sigma, rgb,  \
                                          cap, m_dev)                                              \
           : launch_field_fwd<E, R, false>(s, xyz, bound, table, nullptr, offsets, lv, gridtype,  \
                                           align_corners, w1, b1, w2, b2, w3, b3, enc, sigma, rgb, \
                                           cap, m_dev))
    if (elem == DFHIP_F16 && rgb_dtype == DFHIP_F32) DFHIP_FWD(half_t, float);
    else if (elem == DFHIP_F16 && rgb_dtype == DFHIP_F16) DFHIP_FWD(half_t, half_t);
    else if (elem == DFHIP_BF16 && rgb_dtype == DFHIP_F32) DFHIP_FWD(bf16_t, float);
    else if (elem == DFHIP_BF16 && rgb_dtype == DFHIP_BF16) DFHIP_FWD(bf16_t, bf16_t);
    else {
        set_error("%s: rgb dtype must be f32 or the field's element type", name);
        return DFHIP_EDTYPE;
    }
#undef DFHIP_FWD
    return check_launch(name);
}

extern "C" int dfhip_grid_field_forward(const float *xyz, float bound, const void *table,
                                        const int32_t *offsets, uint32_t L, float S, uint32_t H,
                                        uint32_t gridtype, int align_corners, const float *w1,
                                        const float *b1, const float *w2, const float *b2,
                                        const float *w3, const float *b3, void *enc,
                                        float *sigma, void *rgb, int rgb_dtype, uint32_t cap,
                                        const int32_t *m_dev, dfhip_stream_t stream) {
    return grid_field_forward("grid_field_forward", DFHIP_F16, xyz, bound, table, nullptr,
                              offsets, L, S,
                              H, gridtype, align_corners, w1, b1, w2, b2, w3, b3, enc, sigma,
                              rgb, rgb_dtype, cap, m_dev, stream);
}

extern "C" int dfhip_grid_field_forward_bf16(const float *xyz, float bound, const void *table,
                                             const int32_t *offsets, uint32_t L, float S,
                                             uint32_t H, uint32_t gridtype, int align_corners,
                                             const float *w1, const float *b1, const float *w2,
                                             const float *b2, const float *w3, const float *b3,
                                             void *enc, float *sigma, void *rgb, int rgb_dtype,
                                             uint32_t cap, const int32_t *m_dev,
                                             dfhip_stream_t stream) {
    return grid_field_forward("grid_field_forward_bf16", DFHIP_BF16, xyz, bound, table, nullptr,
                              offsets,
                              L, S, H, gridtype, align_corners, w1, b1, w2, b2, w3, b3, enc,
                              sigma, rgb, rgb_dtype, cap, m_dev, stream);
}

// The autocast table (f32 embeddings rounded to the element type, as
// grid.py:38-39's cast) and its corner quads for QUAD forwards: one thread per
// row; quad entries of hashed / modulo levels and corners past a dense
// level's end (never read: a reachable cell's corners are rows of its level)
// are left zero.
template <typename E>
__global__ __launch_bounds__(256) void k_grid_quads(const float *__restrict__ emb,
                                                    const int32_t *__restrict__ offsets,
                                                    ge::Levels lv, uint32_t gridtype,
                                                    int align_corners, uint32_t rows,
                                                    uint32_t *__restrict__ table,
                                                    u32x4 *__restrict__ quads) {
    __shared__ LevelK LK[kLevels];
    __shared__ uint32_t OFF[kLevels + 1];
    stage_levels(LK, offsets, lv, gridtype, align_corners != 0);
    for (int l = threadIdx.x; l <= kLevels; l += blockDim.x) OFF[l] = (uint32_t)offsets[l];
    __syncthreads();
    const float2 *e2 = reinterpret_cast<const float2 *>(emb);
    auto pack = [&](uint32_t row) {
        const float2 f = e2[row];
        E v[2] = {(E)f.x, (E)f.y};
        uint32_t u;
        __builtin_memcpy(&u, v, 4);
        return u;
    };
    for (uint32_t row = blockIdx.x * blockDim.x + threadIdx.x; row < rows;
         row += gridDim.x * blockDim.x) {
        table[row] = pack(row);
        int l = 0;
        while (l < kLevels - 1 && row >= OFF[l + 1]) ++l;
        const LevelK k = LK[l];
        u32x4 q = {0u, 0u, 0u, 0u};
        if (k.flags == 0u) {
            const uint32_t r = row - k.base, n = OFF[l + 1] - OFF[l];
            const uint32_t o[4] = {0u, 1u, k.m1, k.m1 + 1u};
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const uint32_t idx = (r + o[j]) & k.wmask;
                if (idx < n) q[j] = pack(k.base + idx);
            }
        }
        quads[row] = q;
    }
}

extern "C" int dfhip_grid_quads(int elem, const float *embeddings, const int32_t *offsets,
                                uint32_t L, float S, uint32_t H, uint32_t gridtype,
                                int align_corners, uint32_t rows, void *table, void *quads,
                                dfhip_stream_t stream) {
    const char *name = "grid_quads";
    if (!check_field_grid(name, L)) return DFHIP_EINVAL;
    if (rows == 0) return DFHIP_OK;
    if (!embeddings || !offsets || !table || !quads) {
        set_error("%s: null pointer", name);
        return DFHIP_EINVAL;
    }
    if (((uintptr_t)quads & 15u) != 0) {
        set_error("%s: quads must be 16-byte aligned", name);
        return DFHIP_EINVAL;
    }
    hipStream_t s = as_stream(stream);
    const ge::Levels lv = ge::make_levels(L, S, H);
    const uint32_t blocks = ceil_div(rows, 256u) < 4096u ? ceil_div(rows, 256u) : 4096u;
    if (elem == DFHIP_F16)
        k_grid_quads<half_t><<<blocks, 256, 0, s>>>(embeddings, offsets, lv, gridtype,
                                                     align_corners, rows, (uint32_t *)table,
                                                     (u32x4 *)quads);
    else if (elem == DFHIP_BF16)
        k_grid_quads<bf16_t><<<blocks, 256, 0, s>>>(embeddings, offsets, lv, gridtype,
                                                     align_corners, rows, (uint32_t *)table,
                                                     (u32x4 *)quads);
    else {
        set_error("%s: elem must be f16 or bf16", name);
        return DFHIP_EDTYPE;
    }
    return check_launch(name);
}

// The fused forward reading the corner quads of dfhip_grid_quads (same
// results as dfhip_grid_field_forward[_bf16] on the table made with them).
extern "C" int dfhip_grid_field_forward_quads(int elem, const float *xyz, float bound,
                                              const void *table, const void *quads,
                                              const int32_t *offsets, uint32_t L, float S,
                                              uint32_t H, uint32_t gridtype, int align_corners,
                                              const float *w1, const float *b1, const float *w2,
                                              const float *b2, const float *w3, const float *b3,
                                              void *enc, float *sigma, void *rgb, int rgb_dtype,
                                              uint32_t cap, const int32_t *m_dev,
                                              dfhip_stream_t stream) {
    if (!quads) {
        set_error("grid_field_forward_quads: null quads");
        return DFHIP_EINVAL;
    }
    if (reinterpret_cast<uintptr_t>(quads) & 15) {
        set_error("grid_field_forward_quads: quads must be 16-byte aligned");
        return DFHIP_EINVAL;
    }
    return grid_field_forward("grid_field_forward_quads", elem, xyz, bound, table, quads,
                              offsets, L, S, H, gridtype, align_corners, w1, b1, w2, b2, w3, b3,
                              enc, sigma, rgb, rgb_dtype, cap, m_dev, stream);
}

static int grid_field_backward(
    const char *name, int elem, const void *enc, const float *xyz, float bound, const float *w1,
    const float *b1, const float *w2, const float *b2, const float *w3, const float *b3,
    const float *grad_sigma, const void *grad_rgb, int grad_rgb_dtype, uint32_t cap,
    const int32_t *m_dev, void *d_enc_lbc, float *mlp_partial, uint32_t mlp_parts, float *gw1,
    float *gb1, float *gw2, float *gb2, float *gw3, float *gb3, const int32_t *offsets,
    uint32_t total_rows, uint32_t L, float S, uint32_t H, uint32_t gridtype, int align_corners,
    float *grad_embeddings, float *grid_partial, uint32_t grid_parts, int accumulate,
    dfhip_stream_t stream) {
    if (!check_field_grid(name, L)) return DFHIP_EINVAL;
    if (!(bound > 0.0f)) {
        set_error("%s: bound must be > 0", name);
        return DFHIP_EINVAL;
    }
    if (!w1 || !b1 || !w2 || !b2 || !w3 || !b3 || !gw1 || !gb1 || !gw2 || !gb2 || !gw3 || !gb3 ||
        !mlp_partial) {
        set_error("%s: null pointer", name);
        return DFHIP_EINVAL;
    }
    hipStream_t s = as_stream(stream);
    if (cap > 0) {
        if (!enc || !xyz || !grad_sigma || !grad_rgb || !d_enc_lbc) {
            set_error("%s: null pointer", name);
            return DFHIP_EINVAL;
        }
        if (mlp_parts != bwd_parts(cap)) {
            set_error("%s: mlp_parts must be dfhip_field_mlp_backward_parts(cap) = %u (got %u)",
                      name, bwd_parts(cap), mlp_parts);
            return DFHIP_EINVAL;
        }
        const uint32_t nblk = bwd_blocks(cap);
#define DFHIP_BWD(E, R)                                                                       \
    k_field_bwd<E, R, true><<<nblk, 256, 0, s>>>(                                             \
        (const E *)enc, xyz, w1, b1, w2, b2, w3, b3, grad_sigma, (const R *)grad_rgb, cap,     \
        m_dev, (E *)d_enc_lbc, mlp_partial)
        if (elem == DFHIP_F16 && grad_rgb_dtype == DFHIP_F32) DFHIP_BWD(half_t, float);
        else if (elem == DFHIP_F16 && grad_rgb_dtype == DFHIP_F16) DFHIP_BWD(half_t, half_t);
        else if (elem == DFHIP_BF16 && grad_rgb_dtype == DFHIP_F32) DFHIP_BWD(bf16_t, float);
        else if (elem == DFHIP_BF16 && grad_rgb_dtype == DFHIP_BF16) DFHIP_BWD(bf16_t, bf16_t);
        else {
            set_error("%s: grad_rgb dtype must be f32 or the field's element type", name);
            return DFHIP_EDTYPE;
        }
#undef DFHIP_BWD
    } else {
        mlp_parts = 1;
        (void)hipMemsetAsync(mlp_partial, 0, kParams * sizeof(float), s);
    }
    k_field_wgrad_sum<<<ceil_div((uint32_t)kParams, 64u), 1024, 0, s>>>(
        mlp_partial, mlp_parts, gw1, gb1, gw2, gb2, gw3, gb3, accumulate);
    int rc = check_launch(name);
    if (rc != DFHIP_OK || grad_embeddings == nullptr) return rc;
    if (elem != DFHIP_F16) {
        set_error("%s: the sliced embedding backward takes f16 feature gradients; pass "
                  "grad_embeddings = NULL and use dfhip_grid_encode_backward_binned", name);
        return DFHIP_EDTYPE;
    }
    return ge::grid_backward_sliced(name, DFHIP_F16, DFHIP_F32, d_enc_lbc, xyz, offsets,
                                    grad_embeddings, total_rows, cap, 3, 2, L, S, H, gridtype,
                                    align_corners, grid_partial, grid_parts, accumulate,
                                    ge::SliceDyn{m_dev, bound}, s);
}

extern "C" int dfhip_grid_field_backward(
    const void *enc, const float *xyz, float bound, const float *w1, const float *b1,
    const float *w2, const float *b2, const float *w3, const float *b3, const float *grad_sigma,
    const void *grad_rgb, int grad_rgb_dtype, uint32_t cap, const int32_t *m_dev,
    void *d_enc_lbc, float *mlp_partial, uint32_t mlp_parts, float *gw1, float *gb1, float *gw2,
    float *gb2, float *gw3, float *gb3, const int32_t *offsets, uint32_t total_rows, uint32_t L,
    float S, uint32_t H, uint32_t gridtype, int align_corners, float *grad_embeddings,
    float *grid_partial, uint32_t grid_parts, dfhip_stream_t stream) {
    return grid_field_backward("grid_field_backward", DFHIP_F16, enc, xyz, bound, w1, b1, w2, b2, w3, b3,
                               grad_sigma, grad_rgb, grad_rgb_dtype, cap, m_dev, d_enc_lbc,
                               mlp_partial, mlp_parts, gw1, gb1, gw2, gb2, gw3, gb3, offsets,
                               total_rows, L, S, H, gridtype, align_corners, grad_embeddings,
                               grid_partial, grid_parts, 0, stream);
}

extern "C" int dfhip_grid_field_backward_accumulate(
    const void *enc, const float *xyz, float bound, const float *w1, const float *b1,
    const float *w2, const float *b2, const float *w3, const float *b3, const float *grad_sigma,
    const void *grad_rgb, int grad_rgb_dtype, uint32_t cap, const int32_t *m_dev,
    void *d_enc_lbc, float *mlp_partial, uint32_t mlp_parts, float *gw1, float *gb1, float *gw2,
    float *gb2, float *gw3, float *gb3, const int32_t *offsets, uint32_t total_rows, uint32_t L,
    float S, uint32_t H, uint32_t gridtype, int align_corners, float *grad_embeddings,
    float *grid_partial, uint32_t grid_parts, dfhip_stream_t stream) {
    return grid_field_backward("grid_field_backward_accumulate", DFHIP_F16, enc, xyz, bound, w1, b1, w2, b2,
                               w3, b3, grad_sigma, grad_rgb, grad_rgb_dtype, cap, m_dev, d_enc_lbc,
                               mlp_partial, mlp_parts, gw1, gb1, gw2, gb2, gw3, gb3, offsets,
                               total_rows, L, S, H, gridtype, align_corners, grad_embeddings,
                               grid_partial, grid_parts, 1, stream);
}

extern "C" int dfhip_grid_field_backward_bf16(
    const void *enc, const float *xyz, float bound, const float *w1, const float *b1,
    const float *w2, const float *b2, const float *w3, const float *b3, const float *grad_sigma,
    const void *grad_rgb, int grad_rgb_dtype, uint32_t cap, const int32_t *m_dev,
    void *d_enc_lbc, float *mlp_partial, uint32_t mlp_parts, float *gw1, float *gb1, float *gw2,
    float *gb2, float *gw3, float *gb3, int accumulate, dfhip_stream_t stream) {
    return grid_field_backward("grid_field_backward_bf16", DFHIP_BF16, enc, xyz, bound, w1, b1,
                               w2, b2, w3, b3, grad_sigma, grad_rgb, grad_rgb_dtype, cap, m_dev,
                               d_enc_lbc, mlp_partial, mlp_parts, gw1, gb1, gw2, gb2, gw3, gb3,
                               nullptr, 0, 16, 0.0f, 0, 0, 0, nullptr, nullptr, 0, accumulate,
                               stream);
}
