// Device building blocks of the fused grid field (tiled-grid gather, the
// 32 -> 64 -> 64 -> 4 sigma MLP on v_mfma_f32_16x16x32_f16, the density /
// albedo heads), shared by the train-path kernels (fieldmlp.hip) and the
// fused inference renderer (render.hip).  See fieldmlp.hip for the operand
// maps and the transposed-layer scheme.
#pragma once

#include "common.h"
#include "grid_common.h"

#include <type_traits>

namespace dfhip {
namespace fm {

typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef _Float16 half4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf4 __attribute__((ext_vector_type(4)));
typedef float f4 __attribute__((ext_vector_type(4)));

constexpr int kIn = 32, kHid = 64, kOut = 4;
// packed parameter order (nn.Linear): W1 [64,32], b1 [64], W2 [64,64], b2 [64], W3 [4,64], b3 [4]
constexpr int kOffW1 = 0, kOffB1 = kOffW1 + kHid * kIn, kOffW2 = kOffB1 + kHid,
              kOffB2 = kOffW2 + kHid * kHid, kOffW3 = kOffB2 + kHid, kOffB3 = kOffW3 + kOut * kHid,
              kParams = kOffB3 + kOut;  // 6532

// Field element type T: f16 (the reference's fp16 autocast, C2) or bf16 (the
// C5 option: bf16 autocast, new in this build).  Operand vectors of T and
// the matching gfx950 MFMAs (v_mfma_f32_16x16x32_{f16,bf16}).
typedef _Float16 half2v __attribute__((ext_vector_type(2)));
typedef float f2v __attribute__((ext_vector_type(2)));

template <typename T> struct Elem;
template <> struct Elem<half_t> { typedef half8 v8; typedef half4 v4; };
template <> struct Elem<bf16_t> { typedef bf8 v8; typedef bf4 v4; };
template <typename T> struct Id { typedef T type; };  // non-deduced context

__device__ __forceinline__ f4 mfma(half8 a, half8 b, f4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ f4 mfma(bf8 a, bf8 b, f4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

// Make this wave's LDS writes visible to its other lanes before they read.
__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// LDS row strides (halves).  Operand reads put 16 lanes on 16 consecutive
// rows; a row stride of 4 * odd dwords maps those rows to 16 distinct
// 4-dword bank groups, so the 8-B / 16-B operand reads are conflict-free
// (unpadded 64- and 128-B rows were 4- and 8-way conflicts).
constexpr int kLd32 = 40;  // rows of 32 halves (+8)
constexpr int kLd64 = 72;  // rows of 64 halves (+8)

// Weights as T (autocast's cast of the f32 parameters), in LDS.
template <typename T>
struct WeightsG {
    T w1[kHid * kLd32];  // [n1][f]
    T w2[kHid * kLd64];  // [n2][n1]
    T w3[16 * kLd64];    // [row][n2]: output r in row 4 r (lane group r of the
                         // accumulator tile, element 0), the other rows zero
    float b1[kHid], b2[kHid], b3[16];  // f32 of the T-rounded biases; b3 as w3's rows
};
template <typename T>
struct WeightsTG {       // backward only
    T w1t[kIn * kLd64];  // [f][n1]
    T w2t[kHid * kLd64]; // [n1][n2]
    T w3t[kHid * kLd32]; // [n2][k]: output r at k = 8 r (the B operand's lane group r,
                         // element 0), the other columns zero
};
typedef WeightsG<half_t> Weights;
typedef WeightsTG<half_t> WeightsT;

// Feature order of the fused path: position p = 8h + j of the layer-1 B
// operand holds level 4 (j >> 1) + h, channel j & 1, so that for each j the
// four lane groups work on four levels of the same kind (dense / tiled /
// z-dropped): feature index 2 * level + channel.
__host__ __device__ constexpr int perm_feature(int p) {
    return 2 * (4 * ((p & 7) >> 1) + (p >> 3)) + (p & 1);
}

// PERM: layer-1 weights stored in the fused path's permuted feature order.
template <bool PERM, typename E>
__device__ void load_weights(WeightsG<E> &W, typename Id<WeightsTG<E>>::type *T, const float *w1,
                             const float *b1, const float *w2, const float *b2, const float *w3,
                             const float *b3) {
    for (int i = threadIdx.x; i < kHid * kIn; i += blockDim.x) {
        const int n = i / kIn, p = i % kIn;
        W.w1[n * kLd32 + p] = (E)w1[n * kIn + (PERM ? perm_feature(p) : p)];
        if (T) T->w1t[(i % kIn) * kLd64 + i / kIn] = (E)w1[i];  // natural: rows = features
    }
    for (int i = threadIdx.x; i < kHid * kHid; i += blockDim.x) {
        const E v = (E)w2[i];
        W.w2[(i / kHid) * kLd64 + i % kHid] = v;
        if (T) T->w2t[(i % kHid) * kLd64 + i / kHid] = v;
    }
    for (int i = threadIdx.x; i < 16 * kHid; i += blockDim.x) {
        const int row = i / kHid, n2 = i % kHid;
        W.w3[row * kLd64 + n2] = (row & 3) == 0 ? (E)w3[(row >> 2) * kHid + n2] : (E)0.0f;
    }
    if (T)
        for (int i = threadIdx.x; i < kHid * 32; i += blockDim.x) {
            const int n2 = i / 32, o = i % 32;
            T->w3t[n2 * kLd32 + o] = (o & 7) == 0 ? (E)w3[(o >> 3) * kHid + n2] : (E)0.0f;
        }
    for (int i = threadIdx.x; i < kHid; i += blockDim.x) {
        W.b1[i] = (float)(E)b1[i];
        W.b2[i] = (float)(E)b2[i];
    }
    for (int i = threadIdx.x; i < 16; i += blockDim.x)
        W.b3[i] = (i & 3) == 0 ? (float)(E)b3[i >> 2] : 0.0f;
}

// A operand, natural k order: row `row` of a row-major [*, ld] f16 matrix,
// k = 8h .. 8h+7 (+ koff).
template <typename E>
__device__ __forceinline__ typename Elem<E>::v8 a_nat(const E *m, int ld, int row, int koff, int h) {
    return *reinterpret_cast<const typename Elem<E>::v8 *>(m + row * ld + koff + 8 * h);
}
// A operand, permuted k order of k-step s (see header).
template <typename E>
__device__ __forceinline__ typename Elem<E>::v8 a_perm(const E *m, int ld, int row, int s, int h) {
    typedef typename Elem<E>::v4 v4;
    const v4 lo = *reinterpret_cast<const v4 *>(m + row * ld + 32 * s + 4 * h);
    const v4 hi = *reinterpret_cast<const v4 *>(m + row * ld + 32 * s + 16 + 4 * h);
    return typename Elem<E>::v8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
}
// B operand of k-step s from four accumulator tiles' f16 values v[tile][reg].
template <typename E>
__device__ __forceinline__ typename Elem<E>::v8 b_from_tiles(const E (&v)[4][4], int s) {
    return typename Elem<E>::v8{v[2 * s][0], v[2 * s][1], v[2 * s][2], v[2 * s][3],
                                v[2 * s + 1][0], v[2 * s + 1][1], v[2 * s + 1][2],
                                v[2 * s + 1][3]};
}
// bf16 tiles are kept as packed 4-vectors (two VGPRs each): element-wise
// bf16 scalars cost a VGPR apiece and spilled the forward kernel.
__device__ __forceinline__ bf8 b_from_tiles(const bf4 (&v)[4], int s) {
    return __builtin_shufflevector(v[2 * s], v[2 * s + 1], 0, 1, 2, 3, 4, 5, 6, 7);
}
// Four f32 accumulators -> ReLU -> packed bf16 (relu and round-to-nearest
// commute, so this equals ReLU of the rounded value, autocast's order).
__device__ __forceinline__ bf4 relu_bf4(f4 a) {
    const f4 r = {fmaxf(a[0], 0.0f), fmaxf(a[1], 0.0f), fmaxf(a[2], 0.0f), fmaxf(a[3], 0.0f)};
    return __builtin_convertvector(r, bf4);
}

// Per-tile activations of one layer: [tile][reg] as scalars (f16) or as
// packed vectors (bf16; and f16 with P, the backward: one VGPR per two
// values instead of one per value); all index as t[tile][reg].
template <typename E, bool P = false> struct TilesT { typedef E type[4][4]; };
template <typename E> struct TilesT<E, true> { typedef typename Elem<E>::v4 type[4]; };
template <> struct TilesT<bf16_t, false> { typedef bf4 type[4]; };
template <typename E> struct Tiles : TilesT<E, false> {};
__device__ __forceinline__ half8 b_from_tiles(const half4 (&v)[4], int s) {
    return __builtin_shufflevector(v[2 * s], v[2 * s + 1], 0, 1, 2, 3, 4, 5, 6, 7);
}
__device__ __forceinline__ f4 bias4(const float *b, int row0) {
    return f4{b[row0], b[row0 + 1], b[row0 + 2], b[row0 + 3]};
}

// One 16-sample tile through the MLP.  xb: B operand of the encoder features
// (lane: sample c, features 8h..8h+7).  Outputs the post-ReLU activations (T)
// of both hidden layers and the f32 accumulators of the output layer.
template <typename E, bool P = false>
struct FwdG {
    typename TilesT<E, P>::type a1, a2;  // [tile][reg]: neuron 16 t + 4 h + r of sample c
    f4 o;                                // rows 4h + r: o[0] of lane group h is output h
};
typedef FwdG<half_t> Fwd;

// Four f32 accumulators -> f16 (RNE) -> ReLU as packed f16 pairs (v_cvt_pk
// + v_pk_max: two values per instruction; the same values as the scalar
// form except possibly the sign of a zero, which no product, sum or
// ReLU mask downstream can see unless every term of a sum is zero).
__device__ __forceinline__ half4 relu_h4(f4 a) {
    const half4 v = __builtin_convertvector(a, half4);
    return __builtin_elementwise_max(v, half4{(half_t)0.0f, (half_t)0.0f, (half_t)0.0f,
                                              (half_t)0.0f});
}

// W2R / W1R / W3R: the layer's weight operands come from w2op / w1op / w3op
// (registers, loaded once per kernel) instead of LDS.
template <typename E, bool P, bool W2R = false, bool W1R = false, bool W3R = false>
__device__ __forceinline__ void forward_tile(const WeightsG<E> &W, typename Elem<E>::v8 xb, int c,
                                             int h, FwdG<E, P> &F,
                                             const typename Elem<E>::v8 (*w2op)[2] = nullptr,
                                             const typename Elem<E>::v8 *w1op = nullptr,
                                             const typename Elem<E>::v8 *w3op = nullptr) {
    constexpr bool kBf = std::is_same<E, bf16_t>::value;
    constexpr bool kPkH = P && std::is_same<E, half_t>::value;  // packed f16 (the backward)
    f4 acc[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
        acc[t] = mfma(W1R ? w1op[t] : a_nat(W.w1, kLd32, 16 * t + c, 0, h), xb,
                      bias4(W.b1, 16 * t + 4 * h));
        if constexpr (kBf) {
            F.a1[t] = relu_bf4(acc[t]);
        } else if constexpr (kPkH) {
            F.a1[t] = relu_h4(acc[t]);
        } else {
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const E v = (E)acc[t][r];
                F.a1[t][r] = v > (E)0.0f ? v : (E)0.0f;
            }
        }
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        f4 a = bias4(W.b2, 16 * u + 4 * h);
#pragma unroll
        for (int s = 0; s < 2; ++s)
            a = mfma(W2R ? w2op[u][s] : a_perm(W.w2, kLd64, 16 * u + c, s, h),
                     b_from_tiles(F.a1, s), a);
        if constexpr (kBf) {
            F.a2[u] = relu_bf4(a);
        } else if constexpr (kPkH) {
            F.a2[u] = relu_h4(a);
        } else {
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const E v = (E)a[r];
                F.a2[u][r] = v > (E)0.0f ? v : (E)0.0f;
            }
        }
    }
    f4 o = bias4(W.b3, 4 * h);
#pragma unroll
    for (int s = 0; s < 2; ++s)
        o = mfma(W3R ? w3op[s] : a_perm(W.w3, kLd64, c, s, h), b_from_tiles(F.a2, s), o);
    F.o = o;
}

__device__ __forceinline__ float gaussian(const float *x) {
    // network_grid.py gaussian: 5 * exp(-(x**2).sum(-1) / (2 * 0.2**2)), f32
    const float s = (x[0] * x[0] + x[1] * x[1]) + x[2] * x[2];
    return 5.0f * expf(-s / 0.08f);
}

template <typename E>
__device__ __forceinline__ typename Elem<E>::v8 load_x(const E *enc, uint32_t sample, uint32_t M,
                                                       int h) {
    typedef typename Elem<E>::v8 v8;
    if (sample >= M) return v8{};
    return *reinterpret_cast<const v8 *>(enc + (size_t)sample * kIn + 8 * h);
}

// Per-level constants of the 16-level 3-D grid, staged once per workgroup
// in LDS (the level a lane reads depends on its lane group, so they cannot
// live in scalar registers; reading them from offsets[] / the kernarg Levels
// per tile put dependent global loads in front of every gather).
// Row of corner (p0, p1, p2) = base + wrap(p0 + p1 m1 + p2 m2) with m1 =
// stride of y (0 when the tiled index stops before y), m2 = stride of z (0
// for the z-dropped levels 9-15, gridencoder.cu:56-63); u32 arithmetic as the
// reference's.  wrap: & wmask (power-of-two level, or all-ones for a dense
// level whose index never reaches hsize), or % hsize (flag 1), or the
// spatial hash (flag 2).
struct LevelK {
    uint32_t base, hsize, wmask, m1, m2, flags;
    float scale;
};
constexpr int kLevels = 16;

__device__ __forceinline__ void stage_levels(LevelK *lk, const int32_t *__restrict__ offsets,
                                             const ge::Levels &lv, uint32_t gridtype, bool align) {
    for (int l = threadIdx.x; l < kLevels; l += blockDim.x) {
        const ge::LevelCtx c = ge::level_ctx<3>(offsets, lv, l, gridtype, align);
        LevelK k;
        k.base = c.base;
        k.hsize = c.hsize;
        k.scale = c.scale;
        const uint32_t lead = c.hashed ? 3u : c.used;
        k.m1 = lead > 1 ? c.smul : 0u;
        k.m2 = lead > 2 ? c.smul * c.smul : 0u;
        uint64_t span = 1;  // largest tiled index + 1
        for (uint32_t d = 0; d < c.used; ++d) span *= c.smul;
        k.flags = 0;
        if (c.hashed) {
            k.flags = 2u;
            k.wmask = c.pow2 ? c.hsize - 1u : 0xFFFFFFFFu;
            if (!c.pow2) k.flags |= 1u;
        } else if (c.pow2) {
            k.wmask = c.hsize - 1u;
        } else if (span <= c.hsize) {
            k.wmask = 0xFFFFFFFFu;
        } else {
            k.wmask = 0xFFFFFFFFu;
            k.flags = 1u;
        }
        lk[l] = k;
    }
}

// Grid features of one sample at levels 4(j >> 1) + h (j = 0..7, channel
// j & 1) in the permuted order above.  f16: exactly k_grid_fwd<half, 3, 2>'s
// arithmetic (gridencoder.cu:75-178: half accumulators rounded per corner, in
// corner order).  bf16 (no reference counterpart: its kernels dispatch f32 /
// f16 / f64 only): f32 accumulators, fmaf per corner in corner order, ONE
// rounding to bf16 — per-corner bf16 rounding would lose 3 more bits than the
// f16 path's.  Tiled / dense levels load the corners as four x-neighbour
// pairs (one 8-byte load each; two on z-dropped levels, whose corners 4-7
// are the rows of 0-3): 50 gathers per sample over the 16 levels instead of
// 128, which is what bounds this gather (one scattered lane request per CU
// clock in the L1).  Two levels' loads are issued before their accumulation.
// two table rows (f16 / bf16 pairs) at a 4-byte-aligned address
typedef uint32_t u32x2a __attribute__((ext_vector_type(2), aligned(4)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// QUAD: `quads` (dfhip_grid_quads) holds, for every row r of a tiled / dense
// level, the rows r, r + 1, r + m1, r + m1 + 1 (wrapped like the corners), so
// a level's corners 0-3 are ONE 16-byte load and corners 4-7 another (none on
// a z-dropped level): 25 gathers per sample.  Same values, same order.
template <typename E, bool QUAD = false>
__device__ __forceinline__ typename Elem<E>::v8 grid_features(const E *__restrict__ table,
                                                              const LevelK *lk, bool align,
                                                              const float (&x)[3], int h,
                                                              const u32x4 *__restrict__ quads =
                                                                  nullptr) {
    typename Elem<E>::v8 out{};
    typedef float f8 __attribute__((ext_vector_type(8)));
    f8 outf{};  // bf16: the f32 features, converted to bf16 pairs at the end
    if (x[0] < 0.0f || x[0] > 1.0f || x[1] < 0.0f || x[1] > 1.0f || x[2] < 0.0f || x[2] > 1.0f)
        return out;  // gridencoder.cu:91-100: out-of-range samples encode to zero
    const uint32_t *tab = reinterpret_cast<const uint32_t *>(table);
    // two batches of two levels: up to 8 pair loads in flight per lane per
    // batch (all four levels at once held 64 VGPRs of rows and bits and
    // capped the kernel at 4 waves per SIMD)
#pragma unroll
    for (int half = 0; half < 2; ++half) {
        float frac[2][3];
        uint32_t bits[2][8];
#pragma unroll
        for (int qq = 0; qq < 2; ++qq) {
            const LevelK k = lk[4 * (2 * half + qq) + h];
            uint32_t cell[3];
#pragma unroll
            for (int d = 0; d < 3; ++d) {
                const float p = fmaf(x[d], k.scale, align ? 0.0f : 0.5f);
                cell[d] = (uint32_t)floorf(p);
                frac[qq][d] = p - (float)cell[d];
            }
            if (k.flags == 0u) {
                // tiled / dense: corner offsets {0, 1, m1, m1 + 1, m2, ...}.
                // Corners 2p and 2p + 1 are neighbouring rows unless the
                // wrap falls between them: one 8-byte load per pair.  On a
                // z-dropped level (m2 = 0) corners 4-7 are the rows of 0-3.
                const uint32_t i0 = cell[0] + cell[1] * k.m1 + cell[2] * k.m2;
                const uint32_t ob[4] = {0u, k.m1, k.m2, k.m2 + k.m1};
                const bool zdrop = k.m2 == 0u;
                if constexpr (QUAD) {
                    const u32x4 q0 = quads[k.base + (i0 & k.wmask)];
                    u32x4 q1 = q0;
                    if (!zdrop) q1 = quads[k.base + ((i0 + k.m2) & k.wmask)];
#pragma unroll
                    for (int j = 0; j < 4; ++j) {
                        bits[qq][j] = q0[j];
                        bits[qq][4 + j] = q1[j];
                    }
                    continue;
                }
#pragma unroll
                for (int p = 0; p < 4; ++p) {
                    if (p >= 2 && zdrop) {
                        bits[qq][2 * p] = bits[qq][2 * p - 4];
                        bits[qq][2 * p + 1] = bits[qq][2 * p - 3];
                        continue;
                    }
                    const uint32_t r = (i0 + ob[p]) & k.wmask;
                    const uint32_t *src = tab + k.base + r;
                    if (r != k.wmask) {
                        const u32x2a v = *reinterpret_cast<const u32x2a *>(src);
                        bits[qq][2 * p] = v[0];
                        bits[qq][2 * p + 1] = v[1];
                    } else {
                        bits[qq][2 * p] = src[0];
                        bits[qq][2 * p + 1] = tab[k.base + ((r + 1u) & k.wmask)];
                    }
                }
            } else {
#pragma unroll
                for (uint32_t c = 0; c < 8; ++c) {
                    const uint32_t px = cell[0] + (c & 1u), py = cell[1] + ((c >> 1) & 1u),
                                   pz = cell[2] + ((c >> 2) & 1u);
                    uint32_t idx = (k.flags & 2u) ? (px ^ (py * 2654435761u) ^ (pz * 805459861u))
                                                  : px + py * k.m1 + pz * k.m2;
                    idx = (k.flags & 1u) ? idx % k.hsize : (idx & k.wmask);
                    bits[qq][c] = tab[k.base + idx];
                }
            }
        }
#pragma unroll
        for (int qq = 0; qq < 2; ++qq) {
            // f16: half accumulators (the reference's scalar_t); bf16: f32
            typedef typename std::conditional<std::is_same<E, half_t>::value, half_t, float>::type
                acc_t;
            acc_t a0 = (acc_t)0.0f, a1 = (acc_t)0.0f;
            // f16: both channels at once, c10::Half's two roundings per corner:
            // p = Half(w * float(g)) as v_pk_mul_f32 + v_cvt_pk_f16_f32 (the
            // value barrier keeps them from fusing into one rounding), then
            // r = Half(float(r) + float(p)) as v_pk_add_f16 — f32 holds
            // 24 >= 2 x 11 + 2 bits, so rounding the f32 sum again to f16
            // equals the correctly rounded f16 add (double rounding is
            // innocuous at that precision)
            half2v acc2 = half2v{(half_t)0.0f, (half_t)0.0f};
#pragma unroll
            for (uint32_t c = 0; c < 8; ++c) {
                float w = 1.0f;
#pragma unroll
                for (int d = 0; d < 3; ++d) w *= (c & (1u << d)) ? frac[qq][d] : 1.0f - frac[qq][d];
                E v[2];
                __builtin_memcpy(v, &bits[qq][c], 4);
                if constexpr (std::is_same<E, half_t>::value) {
                    f2v prod = f2v{w, w} * f2v{(float)v[0], (float)v[1]};
                    asm("" : "+v"(prod));
                    acc2 += __builtin_convertvector(prod, half2v);
                } else {
                    a0 = fmaf(w, (float)v[0], a0);
                    a1 = fmaf(w, (float)v[1], a1);
                }
            }
            if constexpr (std::is_same<E, half_t>::value) {
                a0 = acc2[0];
                a1 = acc2[1];
            }
            const int q = 2 * half + qq;
            if constexpr (std::is_same<E, half_t>::value) {
                out[2 * q] = a0;
                out[2 * q + 1] = a1;
            } else {
                outf[2 * q] = a0;
                outf[2 * q + 1] = a1;
            }
        }
    }
    if constexpr (!std::is_same<E, half_t>::value) out = __builtin_convertvector(outf, bf8);
    return out;
}

__device__ __forceinline__ uint32_t active_count(const int32_t *m_dev, uint32_t cap) {
    if (!m_dev) return cap;
    const int32_t m = *m_dev;
    return m < 0 ? 0u : ((uint32_t)m < cap ? (uint32_t)m : cap);
}

}  // namespace fm
}  // namespace dfhip
