// wave_simd.hpp — explicit wave64 vector values for the register-resident engine (reg_engine.hpp).
//
// The register engine is written as ONE uniform (scalar) program that manipulates whole-wave
// vectors: V is one 32-bit value per lane (a VGPR), B one predicate per lane (an SGPR-pair mask),
// VA<N> an array of N VGPRs indexed by a wave-uniform index (s_set_gpr_idx on gfx950). All control
// flow depends on scalars only, so the same source has two backends:
//   * the device backend (default): V is a plain per-lane u32, the lane is implicit, cross-lane
//     operations are DPP / ds_bpermute / v_readlane / v_writelane;
//   * the CPU backend (MTE_CPU, test infrastructure only: tests/native/): V holds all 64 lanes and
//     every operation loops over them with the SAME semantics, so the engine's logic is checked
//     against the oracle in the CPU suite. The product path never uses it.
#pragma once
#include <stdint.h>

#ifndef MTE_CPU
#include <hip/hip_runtime.h>
#endif

// lambdas inside the engine must inline like its __forceinline__ members (an outlined closure puts
// every captured register value on the scratch stack)
#define MTE_LI __attribute__((always_inline))

namespace mte {
namespace simd {

typedef uint32_t u32;
typedef int32_t i32;
typedef uint64_t u64;

#ifndef MTE_CPU
// ------------------------------------------------------------------------------- device backend
#define SD __device__ __forceinline__

struct V {
    u32 x;
};
#ifndef MTE_B_MASK
#define MTE_B_MASK 1
#endif
#if MTE_B_MASK
// A per-lane predicate as the wave's 64-bit lane mask (an SGPR pair): a compare is one v_cmp writing
// the pair, &, | and ~ are one SALU op each, sel is one v_cndmask reading the pair
// (inverse_ballot) and ballot is free. (A 0/1 value per lane made every ballot of a combined
// predicate a v_cndmask 0/1 + v_cmp pair.) The program runs with all 64 lanes active.
struct B {
    u64 m;
};
SD B mk(bool c) { return {__builtin_amdgcn_ballot_w64(c)}; }
SD bool lane_of(B c) { return __builtin_amdgcn_inverse_ballot_w64(c.m); }
SD B mk_all() { return {~0ull}; }
SD B mk_none() { return {0ull}; }
#else
struct B {  // a per-lane predicate; u32 0/1 rather than bool: an i1 member defeats SROA (stores i1,
    u32 b;  // loads i8) and left every predicate of the engine on the scratch stack
};
SD B mk(bool c) { return {(u32)c}; }
SD bool lane_of(B c) { return c.b != 0; }
SD B mk_all() { return {1u}; }
SD B mk_none() { return {0u}; }
#endif

SD V lanes() { return V{__lane_id()}; }
SD V splat(u32 s) { return V{s}; }

SD V operator+(V a, V b) { return {a.x + b.x}; }
SD V operator+(V a, u32 b) { return {a.x + b}; }
SD V operator-(V a, V b) { return {a.x - b.x}; }
SD V operator-(V a, u32 b) { return {a.x - b}; }
SD V operator-(u32 a, V b) { return {a - b.x}; }
SD V operator&(V a, V b) { return {a.x & b.x}; }
SD V operator&(V a, u32 b) { return {a.x & b}; }
SD V operator|(V a, V b) { return {a.x | b.x}; }
SD V operator|(V a, u32 b) { return {a.x | b}; }
SD V operator^(V a, u32 b) { return {a.x ^ b}; }
SD V operator*(V a, u32 b) { return {a.x * b}; }
SD V operator<<(V a, u32 s) { return {a.x << s}; }
SD V operator>>(V a, u32 s) { return {a.x >> s}; }
SD V operator>>(V a, V s) { return {a.x >> s.x}; }
SD V shl(V a, V s) { return {a.x << (s.x & 31u)}; }  // per-lane shift count (low 5 bits, as v_lshlrev)
SD V bfe(V a, u32 off, u32 w) { return {__builtin_amdgcn_ubfe(a.x, off, w)}; }

// unsigned compares
SD B operator==(V a, V b) { return mk(a.x == b.x); }
SD B operator==(V a, u32 b) { return mk(a.x == b); }
SD B operator!=(V a, u32 b) { return mk(a.x != b); }
SD B operator<(V a, u32 b) { return mk(a.x < b); }
SD B operator<(V a, V b) { return mk(a.x < b.x); }
SD B operator>=(V a, u32 b) { return mk(a.x >= b); }
SD B operator>=(V a, V b) { return mk(a.x >= b.x); }
SD B operator>(V a, u32 b) { return mk(a.x > b); }
// signed compares
SD B slt(V a, V b) { return mk((i32)a.x < (i32)b.x); }
SD B sle(V a, i32 b) { return mk((i32)a.x <= b); }
SD B sgt(V a, i32 b) { return mk((i32)a.x > b); }
SD B sge(V a, i32 b) { return mk((i32)a.x >= b); }
SD B slt(V a, i32 b) { return mk((i32)a.x < b); }
SD B slt(i32 a, V b) { return mk(a < (i32)b.x); }

#if MTE_B_MASK
SD B operator&(B a, B b) { return {a.m & b.m}; }
SD B operator|(B a, B b) { return {a.m | b.m}; }
SD B operator~(B a) { return {~a.m}; }
SD B andn(B a, B b) { return {a.m & ~b.m}; }
SD u64 ballot(B c) { return c.m; }
SD B ballot_mask(u64 m) { return {m}; }
#else
SD B operator&(B a, B b) { return {a.b & b.b}; }
SD B operator|(B a, B b) { return {a.b | b.b}; }
SD B operator~(B a) { return {a.b ^ 1u}; }
SD B andn(B a, B b) { return {a.b & (b.b ^ 1u)}; }
SD u64 ballot(B c) { return __ballot(c.b != 0); }
// the per-lane predicate of a uniform 64-bit mask (lane l: bit l)
SD B ballot_mask(u64 m) { return {(u32)((m >> __lane_id()) & 1ull)}; }
#endif

SD V sel(B c, V a, V b) { return {lane_of(c) ? a.x : b.x}; }
SD V sel(B c, u32 a, V b) { return {lane_of(c) ? a : b.x}; }
SD V sel(B c, V a, u32 b) { return {lane_of(c) ? a.x : b}; }

SD u32 readlane(V v, u32 l) { return __builtin_amdgcn_readlane(v.x, l); }
// v_writelane_b32 through the LLVM intrinsic (this clang has no __builtin for it)
extern "C" __device__ int mte_llvm_writelane(int, int, int) __asm("llvm.amdgcn.writelane.i32");
SD V writelane(V v, u32 l, u32 s) { return {(u32)mte_llvm_writelane((int)s, (int)l, (int)v.x)}; }
// v from lane src[l] for every lane l (ds_bpermute: LDS crossbar, no LDS memory)
SD V bperm(V v, V src) { return {(u32)__builtin_amdgcn_ds_bpermute((int)(src.x << 2), (int)v.x)}; }
// lane l's v to lane dst[l] (ds_permute; dst must be a permutation of the lanes)
SD V push(V v, V dst) { return {(u32)__builtin_amdgcn_ds_permute((int)(dst.x << 2), (int)v.x)}; }
SD V bcnt(V v) { return {(u32)__builtin_popcount(v.x)}; }

// Inclusive prefix sum over the 64 lanes (DPP row_shr 1/2/4/8, row_bcast 15/31).
SD V scan_incl(V v) {
    u32 x = v.x, t;
    t = __builtin_amdgcn_update_dpp(0u, x, 0x111, 0xf, 0xf, false); x += t;
    t = __builtin_amdgcn_update_dpp(0u, x, 0x112, 0xf, 0xf, false); x += t;
    t = __builtin_amdgcn_update_dpp(0u, x, 0x114, 0xf, 0xf, false); x += t;
    t = __builtin_amdgcn_update_dpp(0u, x, 0x118, 0xf, 0xf, false); x += t;
    t = __builtin_amdgcn_update_dpp(0u, x, 0x142, 0xa, 0xf, false); x += t;
    t = __builtin_amdgcn_update_dpp(0u, x, 0x143, 0xc, 0xf, false); x += t;
    return {x};
}
// Sum of each aligned 8-lane group, in every lane of the group: half-row mirror, then two quad
// permutes (no lane ever reads outside its group).
SD V g8_sum(V v) {
    u32 x = v.x;
    x += __builtin_amdgcn_update_dpp(0u, x, 0x141, 0xf, 0xf, false);  // row_half_mirror
    x += __builtin_amdgcn_update_dpp(0u, x, 0x4E, 0xf, 0xf, false);   // quad_perm [2,3,0,1]
    x += __builtin_amdgcn_update_dpp(0u, x, 0xB1, 0xf, 0xf, false);   // quad_perm [1,0,3,2]
    return {x};
}
// Lane l takes lane l-1 inside its 16-lane row (lane 0 of a row takes 0). Used with a mask whose
// lanes never sit at a group start, so no value crosses an 8-lane group.
SD V row_shr1(V v) { return {(u32)__builtin_amdgcn_update_dpp(0u, v.x, 0x111, 0xf, 0xf, false)}; }
// Lane l takes lane l-1 across the whole wave (lane 0 takes 0): DPP wave_shr:1.
SD V wave_shr1(V v) { return {(u32)__builtin_amdgcn_update_dpp(0u, v.x, 0x138, 0xf, 0xf, false)}; }

// N VGPRs indexed by a wave-uniform index (s_set_gpr_idx_on ... v_mov ... off on gfx950).
template <int N>
struct VA {
    typedef u32 vec __attribute__((ext_vector_type(N)));
    vec a;
    SD V get(u32 i) const { return V{a[i]}; }
    SD void set(u32 i, V v) { a[i] = v.x; }
    SD void zero() {
#pragma unroll
        for (int i = 0; i < N; i++) a[i] = 0u;
    }
};

// per-lane memory access (global)
template <class T>
SD V ld(const T* p, V idx, B m) {
    return V{lane_of(m) ? (u32)p[idx.x] : 0u};
}
template <class T>
SD void st(T* p, V idx, V v, B m) {
    if (lane_of(m)) p[idx.x] = (T)v.x;
}
// true in exactly one lane (the lane that performs a wave's single store / atomic)
SD bool lane0() { return __lane_id() == 0; }
// LDS hand-offs between the lanes of one wave: LDS instructions of a wave execute in order, so only
// compiler reordering has to be prevented (no wait, no cache maintenance)
SD void lds_order() {
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
    __builtin_amdgcn_wave_barrier();
}
// Order this wave's earlier global writes before its later global reads by OTHER lanes.
SD void wave_fence() {
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
    __builtin_amdgcn_wave_barrier();
}

#else
// ---------------------------------------------------------------------------------- CPU backend
#define SD inline

struct V {
    u32 x[64];
};
struct B {
    u64 m;
};
SD B mk_all() { return {~0ull}; }
SD B mk_none() { return {0ull}; }
#define MTE_L for (u32 l = 0; l < 64; l++)

SD V lanes() {
    V r;
    MTE_L r.x[l] = l;
    return r;
}
SD V splat(u32 s) {
    V r;
    MTE_L r.x[l] = s;
    return r;
}
#define MTE_VOP(OP)                               \
    SD V operator OP(V a, V b) {                  \
        V r;                                      \
        MTE_L r.x[l] = a.x[l] OP b.x[l];          \
        return r;                                 \
    }                                             \
    SD V operator OP(V a, u32 b) {                \
        V r;                                      \
        MTE_L r.x[l] = a.x[l] OP b;               \
        return r;                                 \
    }
MTE_VOP(+)
MTE_VOP(-)
MTE_VOP(&)
MTE_VOP(|)
MTE_VOP(^)
MTE_VOP(*)
#undef MTE_VOP
SD V operator-(u32 a, V b) {
    V r;
    MTE_L r.x[l] = a - b.x[l];
    return r;
}
SD V operator<<(V a, u32 s) {
    V r;
    MTE_L r.x[l] = s >= 32 ? 0u : a.x[l] << s;
    return r;
}
SD V operator>>(V a, u32 s) {
    V r;
    MTE_L r.x[l] = s >= 32 ? 0u : a.x[l] >> s;
    return r;
}
SD V operator>>(V a, V s) {
    V r;
    MTE_L r.x[l] = a.x[l] >> (s.x[l] & 31);
    return r;
}
SD V shl(V a, V s) {
    V r;
    MTE_L r.x[l] = a.x[l] << (s.x[l] & 31);
    return r;
}
SD V bfe(V a, u32 off, u32 w) {
    V r;
    MTE_L r.x[l] = (a.x[l] >> off) & (w >= 32 ? 0xFFFFFFFFu : ((1u << w) - 1u));
    return r;
}
#define MTE_CMP(NAME, EXPR)                       \
    SD B NAME {                                   \
        B r{0};                                   \
        MTE_L if (EXPR) r.m |= 1ull << l;         \
        return r;                                 \
    }
MTE_CMP(operator==(V a, V b), a.x[l] == b.x[l])
MTE_CMP(operator==(V a, u32 b), a.x[l] == b)
MTE_CMP(operator!=(V a, u32 b), a.x[l] != b)
MTE_CMP(operator<(V a, u32 b), a.x[l] < b)
MTE_CMP(operator<(V a, V b), a.x[l] < b.x[l])
MTE_CMP(operator>=(V a, u32 b), a.x[l] >= b)
MTE_CMP(operator>=(V a, V b), a.x[l] >= b.x[l])
MTE_CMP(operator>(V a, u32 b), a.x[l] > b)
MTE_CMP(slt(V a, V b), (i32)a.x[l] < (i32)b.x[l])
MTE_CMP(sle(V a, i32 b), (i32)a.x[l] <= b)
MTE_CMP(sgt(V a, i32 b), (i32)a.x[l] > b)
MTE_CMP(sge(V a, i32 b), (i32)a.x[l] >= b)
MTE_CMP(slt(V a, i32 b), (i32)a.x[l] < b)
MTE_CMP(slt(i32 a, V b), a < (i32)b.x[l])
#undef MTE_CMP
SD B operator&(B a, B b) { return {a.m & b.m}; }
SD B operator|(B a, B b) { return {a.m | b.m}; }
SD B operator~(B a) { return {~a.m}; }
SD B andn(B a, B b) { return {a.m & ~b.m}; }

SD V sel(B c, V a, V b) {
    V r;
    MTE_L r.x[l] = ((c.m >> l) & 1) ? a.x[l] : b.x[l];
    return r;
}
SD V sel(B c, u32 a, V b) { return sel(c, splat(a), b); }
SD V sel(B c, V a, u32 b) { return sel(c, a, splat(b)); }

SD u64 ballot(B c) { return c.m; }
SD B ballot_mask(u64 m) { return {m}; }
SD u32 readlane(V v, u32 l) { return v.x[l & 63]; }
SD V writelane(V v, u32 l, u32 s) {
    v.x[l & 63] = s;
    return v;
}
SD V bperm(V v, V src) {
    V r;
    MTE_L r.x[l] = v.x[src.x[l] & 63];
    return r;
}
SD V push(V v, V dst) {
    V r;
    bool hit[64] = {false};
    MTE_L {
        const u32 d = dst.x[l] & 63;
        if (hit[d]) __builtin_trap();  // not a permutation
        hit[d] = true;
        r.x[d] = v.x[l];
    }
    return r;
}
SD V bcnt(V v) {
    V r;
    MTE_L r.x[l] = (u32)__builtin_popcount(v.x[l]);
    return r;
}
SD V scan_incl(V v) {
    V r;
    u32 s = 0;
    MTE_L r.x[l] = (s += v.x[l]);
    return r;
}
SD V g8_sum(V v) {
    V r;
    for (u32 g = 0; g < 8; g++) {
        u32 s = 0;
        for (u32 i = 0; i < 8; i++) s += v.x[g * 8 + i];
        for (u32 i = 0; i < 8; i++) r.x[g * 8 + i] = s;
    }
    return r;
}
SD V row_shr1(V v) {
    V r;
    MTE_L r.x[l] = (l & 15) ? v.x[l - 1] : 0u;
    return r;
}
SD V wave_shr1(V v) {
    V r;
    MTE_L r.x[l] = l ? v.x[l - 1] : 0u;
    return r;
}

template <int N>
struct VA {
    V a[N];
    SD V get(u32 i) const { return a[i]; }
    SD void set(u32 i, V v) { a[i] = v; }
    SD void zero() {
        for (int i = 0; i < N; i++) a[i] = splat(0);
    }
};

template <class T>
SD V ld(const T* p, V idx, B m) {
    V r;
    MTE_L r.x[l] = ((m.m >> l) & 1) ? (u32)p[idx.x[l]] : 0u;
    return r;
}
template <class T>
SD void st(T* p, V idx, V v, B m) {
    MTE_L if ((m.m >> l) & 1) p[idx.x[l]] = (T)v.x[l];
}
SD void wave_fence() {}
SD void lds_order() {}
SD bool lane0() { return true; }  // the emulated wave performs a single store once
#undef MTE_L
#endif

}  // namespace simd
}  // namespace mte
