// icp4r_device.hpp — device-side helpers shared by the kernel translation units
// (icp4r_kernels.hip, icp4r_gicp.hip): scalar-cache pointers, the XCD-aware work mapping, the
// slotted work counters and the NN key.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "icp4r_internal.hpp"

namespace icp4r {

using v4f = float __attribute__((ext_vector_type(4)));
// Target pointers are re-typed into the AMDGPU constant address space (4): with a wave-uniform
// address every load becomes an s_load (scalar cache -> SGPRs) whatever alias analysis can prove.
using cv4f_ptr = const __attribute__((address_space(4))) v4f*;

// The address is also made PROVABLY wave-uniform (readfirstlane of both halves, once), so hipcc
// keeps it in SGPRs instead of re-reading it with v_readfirstlane inside the sweep loop.
__device__ __forceinline__ cv4f_ptr as_const(const float4* p) {
    const uint64_t a = reinterpret_cast<uint64_t>(p);
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
    return reinterpret_cast<cv4f_ptr>(((uint64_t)hi << 32) | lo);
}

// Wave-uniform scalar reads of per-pair metadata (read-only during a launch) via s_load, so counts,
// offsets and loop bounds stay in SGPRs.
template <typename T>
__device__ __forceinline__ T uload(const T* p) {
    return *reinterpret_cast<const __attribute__((address_space(4))) T*>(reinterpret_cast<uintptr_t>(p));
}

// XCD-aware work mapping.  Workgroups are dispatched round-robin over the 8 XCDs (linear id mod 8),
// each with its own L2.  Remap linear id L of `total` so that XCD x receives the contiguous work
// range [x*per + min(x, rem), ...): every workgroup of a pair then runs on one XCD, and a pair's
// target index / correspondence records are fetched into one L2 instead of eight.
constexpr int kXcds = 8;
__device__ __forceinline__ int xcd_remap(int L, int total) {
    const int per = total / kXcds, rem = total % kXcds;
    const int xcd = L % kXcds, slot = L / kXcds;
    return xcd * per + min(xcd, rem) + slot;
}

// Work counters: add v to counter k of this wave's slot.  Call from one lane.
__device__ __forceinline__ void count_add(unsigned long long* ctr, int k, unsigned long long v) {
    if (v == 0 || ctr == nullptr) return;  // (null: counting off — WorkArgs::evals)
    const uint32_t blk = blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z);
    const uint32_t slot = (blk * (blockDim.x >> 6) + (threadIdx.x >> 6)) % kCountSlots;
    atomicAdd(ctr + (size_t)slot * kCountStride + k, v);
}

__device__ __forceinline__ NNKey make_key(float d2, uint32_t idx) {
    return ((NNKey)__float_as_uint(d2) << 32) | idx;
}

// A first-pass seed key (src_order_kernel): d² = +inf and an index inside the target (anything else
// in nn_key before the first pass is stale and ignored).
__device__ __forceinline__ bool seed_key(NNKey k, int m) {
    return (uint32_t)(k >> 32) == 0x7f800000u && (uint32_t)k < (uint32_t)m;
}

// Wave-wide float min / max through DPP (no LDS round trip: __shfl_xor compiles to ds_bpermute /
// ds_swizzle, one dependent LDS-unit op per step).  Steps: xor 1 and xor 2 (quad_perm), the 8- and
// 16-lane mirrors, then row_bcast15 / row_bcast31 fold rows 0-1 and 0-3 into row 3; lane 63 holds
// the result, broadcast with readlane.  Every lane of the wave must be active.
template <int CTRL, int ROWS = 0xf>
__device__ __forceinline__ float dpp_f(float v) {
    return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(__builtin_bit_cast(int, v), __builtin_bit_cast(int, v),
                                                                 CTRL, ROWS, 0xf, false));
}
__device__ __forceinline__ float wave_minf(float x) {
    x = fminf(x, dpp_f<0xB1>(x));        // quad_perm [1,0,3,2]
    x = fminf(x, dpp_f<0x4E>(x));        // quad_perm [2,3,0,1]
    x = fminf(x, dpp_f<0x141>(x));       // row_half_mirror
    x = fminf(x, dpp_f<0x140>(x));       // row_mirror
    x = fminf(x, dpp_f<0x142, 0xa>(x));  // row_bcast15 -> rows 1, 3
    x = fminf(x, dpp_f<0x143, 0xc>(x));  // row_bcast31 -> rows 2, 3
    return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, x), 63));
}
// Min / max over each aligned group of B lanes (B = 16: the DPP quad xors and the half-row and row
// mirrors leave every lane of a 16-lane row holding the row's extreme; B = 32 adds one xor-16
// shuffle).  Replaces a __shfl_xor butterfly whose ds_bpermute per step went through the LDS unit
// (the index's block boxes: 6 values x 4 steps per 64 points).  Every lane of the wave active.
__device__ __forceinline__ float seg_minf(float x, int B) {
    x = fminf(x, dpp_f<0xB1>(x));
    x = fminf(x, dpp_f<0x4E>(x));
    x = fminf(x, dpp_f<0x141>(x));
    x = fminf(x, dpp_f<0x140>(x));
    if (B > 16) x = fminf(x, __shfl_xor(x, 16, 64));
    return x;
}
__device__ __forceinline__ float seg_maxf(float x, int B) {
    x = fmaxf(x, dpp_f<0xB1>(x));
    x = fmaxf(x, dpp_f<0x4E>(x));
    x = fmaxf(x, dpp_f<0x141>(x));
    x = fmaxf(x, dpp_f<0x140>(x));
    if (B > 16) x = fmaxf(x, __shfl_xor(x, 16, 64));
    return x;
}

// Inclusive wave prefix sum by DPP (Hillis-Steele inside each 16-lane row by row_shr 1, 2, 4, 8 with
// zero fill, then the row totals carried by row_bcast15 into rows 1, 3 and row_bcast31 into rows
// 2, 3).  Integer adds: exact, the same values as the __shfl_up ladder it replaces, without its six
// dependent ds_bpermute round trips through the LDS unit (the kd builds run one per level).  Every
// lane of the wave active.
template <int CTRL, int ROWS = 0xf>
__device__ __forceinline__ uint32_t dpp_z(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, CTRL, ROWS, 0xf, true);
}
__device__ __forceinline__ uint32_t wave_scan_incl(uint32_t x) {
    x += dpp_z<0x111>(x);       // row_shr:1
    x += dpp_z<0x112>(x);       // row_shr:2
    x += dpp_z<0x114>(x);       // row_shr:4
    x += dpp_z<0x118>(x);       // row_shr:8
    x += dpp_z<0x142, 0xa>(x);  // row_bcast15 -> rows 1, 3
    x += dpp_z<0x143, 0xc>(x);  // row_bcast31 -> rows 2, 3
    return x;
}

// Wave-wide integer sum by the same DPP steps (exact in any order).  No lane addresses: the
// __shfl_xor butterfly's ds_bpermute addresses, shared by the compiler across a kernel's reductions,
// were kept live — and spilled — from pass A's count to the fused test's (fold_update_kernel).
template <int CTRL, int ROWS = 0xf>
__device__ __forceinline__ int dpp_i(int v) {
    return __builtin_amdgcn_update_dpp(v, v, CTRL, ROWS, 0xf, false);
}
__device__ __forceinline__ int wave_sumi(int x) {
    x += dpp_i<0xB1>(x);
    x += dpp_i<0x4E>(x);
    x += dpp_i<0x141>(x);
    x += dpp_i<0x140>(x);
    x += dpp_i<0x142, 0xa>(x);
    x += dpp_i<0x143, 0xc>(x);
    return __builtin_amdgcn_readlane(x, 63);
}
__device__ __forceinline__ float wave_maxf(float x) {
    x = fmaxf(x, dpp_f<0xB1>(x));
    x = fmaxf(x, dpp_f<0x4E>(x));
    x = fmaxf(x, dpp_f<0x141>(x));
    x = fmaxf(x, dpp_f<0x140>(x));
    x = fmaxf(x, dpp_f<0x142, 0xa>(x));
    x = fmaxf(x, dpp_f<0x143, 0xc>(x));
    return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, x), 63));
}

// Write-through stores (experiment, ICP4R_WT bit mask: 1 = the fused test's stores, 2 = the batched
// search's result stores, 4 = the one-tile search's stores: X, keys, correspondence records): `sc1` vector stores leave no dirty line in the XCD's L2, so the kernel
// boundary has less to write back (MI355X_MICROARCH.md §kernel boundary: + dirty bytes / 6 TB/s).
#ifndef ICP4R_WT
#define ICP4R_WT 0
#endif
template <int BIT>
__device__ __forceinline__ void st_v4(float4* p, const float4 v) {
    if constexpr ((ICP4R_WT & BIT) != 0) {
        const v4f x = {v.x, v.y, v.z, v.w};
        asm volatile("global_store_dwordx4 %0, %1, off sc1\n\ts_nop 1" ::"v"(p), "v"(x) : "memory");
    } else {
        *p = v;
    }
}
template <int BIT, typename T>
__device__ __forceinline__ void st_sc(T* p, const T v) {  // 4 or 8 bytes
    if constexpr ((ICP4R_WT & BIT) != 0)
        __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    else
        *p = v;
}

// Box pruning is conservative in float: a box lower bound is shrunk by 2^-16 before its `<=` test
// against a d², which covers the few-ulp rounding of both the bound and l2_simple.
constexpr float kLbShrink = 1.0f - 1.0f / 65536.0f;

}  // namespace icp4r
