// Test-only probe for tools/isa_hazard_check.py (tests/test_isa_hazards.py):
// the product's untracked register load (ld_buf_untracked) and fence
// (reg_fence) used correctly once, and twice with a deliberately injected
// early touch of the destination registers -- the miscompile class the audit
// exists to catch.  Compiled to ISA only; never launched.
#include "../../ggml-cuda-experiments_amd/csrc/fattn_split.h"

using namespace fattn;
typedef float pf32x16 __attribute__((ext_vector_type(16)));

// correct: load, wait, fence, use
__global__ void probe_clean(const uint8_t* p, uint32_t* out, uint32_t bytes) {
    const i32x4 srd = make_srd(p, bytes);
    u32x4 v = ld_buf_untracked<kTagQ>(srd, threadIdx.x * 16);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    reg_fence<kTagQ>(v);
    out[threadIdx.x] = v.x + v.y + v.z + v.w;
}

// injected: the value is stored before its wait (a read of a pending register)
__global__ void probe_early_store(const uint8_t* p, uint32_t* out, uint32_t bytes) {
    const i32x4 srd = make_srd(p, bytes);
    u32x4 v = ld_buf_untracked<kTagQ>(srd, threadIdx.x * 16);
    out[threadIdx.x + 256] = v.y;  // before the wait: stale register contents
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    reg_fence<kTagQ>(v);
    out[threadIdx.x] = v.x;
}

// injected: an early register copy, as hipcc made them in round 3, with a
// counted (not vmcnt(0)) wait -- only the fence retires the load
__global__ void probe_early_copy(const uint8_t* p, uint32_t* out, uint32_t bytes) {
    const i32x4 srd = make_srd(p, bytes);
    u32x4 v = ld_buf_untracked<kTagMaskWords>(srd, threadIdx.x * 16);
    uint32_t c;
    asm volatile("v_mov_b32 %0, %1" : "=v"(c) : "v"(v.z));  // the copy, before the wait
    asm volatile("s_waitcnt vmcnt(1)" ::: "memory");
    reg_fence<kTagMaskWords>(v);
    out[threadIdx.x] = v.x + c;
}

// wait states the compiler cannot see (the checker's second audit): an asm
// v_add_f32 reading a v_exp_f32 result the compiler placed right before it --
// fattn_pf4.h's round-5 row sums -- and the same with the pad inside the asm
__global__ void probe_trans_asm_use(const float* x, float* out) {
    const float v = x[threadIdx.x];
    const float e = __builtin_amdgcn_exp2f(v);
    float r;
    asm volatile("v_add_f32_e32 %0, %1, %2" : "=v"(r) : "v"(v), "v"(e));
    out[threadIdx.x] = r;
}
__global__ void probe_trans_asm_padded(const float* x, float* out) {
    const float v = x[threadIdx.x];
    const float e = __builtin_amdgcn_exp2f(v);
    float r;
    asm volatile("s_nop 0\n\tv_add_f32_e32 %0, %1, %2" : "=v"(r) : "v"(v), "v"(e));
    out[threadIdx.x] = r;
}

// XDL MFMA result -> asm read (the checker's third audit, round 6): a
// 32x32x16 MFMA's accumulator read only by an asm v_accvgpr_read behind a
// branch (fattn_pf4.h's scale_acc16 in the rescale path, without its s_nop
// pad) -- hipcc pads its own reads, not the asm's -- and the same with the pad
__global__ void probe_xdl_asm_read(const f16x8* a, float* out, int flag) {
    pf32x16 acc = {};
    acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[threadIdx.x], a[threadIdx.x + 64], acc, 0, 0, 0);
    float t = 0.0f;
    if (__builtin_amdgcn_readfirstlane(flag)) asm volatile("v_accvgpr_read_b32 %0, %1" : "=v"(t) : "a"(acc[0]));
    out[threadIdx.x] = t;
}
__global__ void probe_xdl_asm_read_padded(const f16x8* a, float* out, int flag) {
    pf32x16 acc = {};
    acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[threadIdx.x], a[threadIdx.x + 64], acc, 0, 0, 0);
    float t = 0.0f;
    if (__builtin_amdgcn_readfirstlane(flag))
        asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7\n\tv_accvgpr_read_b32 %0, %1" : "=v"(t) : "a"(acc[0]));
    out[threadIdx.x] = t;
}

// asm XDL MFMA result -> hipcc's read of it (the third audit's other half,
// round 6): an asm accumulate chain into VGPRs (fattn_pf4.h's lean S^T
// chains) whose result hipcc's code reads at once -- hipcc pads only its own
// MFMAs -- and the same chain ending in the 12 states of a 32x32x16 MFMA (the
// chain's second step takes the first's result whole as srcC: no wait)
__global__ void probe_xdl_vgpr_read(const f16x8* a, float* out) {
    pf32x16 acc;
    asm volatile("v_mfma_f32_32x32x16_f16 %0, %1, %2, 0" : "=&v"(acc) : "v"(a[threadIdx.x]), "v"(a[threadIdx.x + 64]));
    asm volatile("v_mfma_f32_32x32x16_f16 %0, %1, %2, %0" : "+v"(acc) : "v"(a[threadIdx.x + 128]), "v"(a[threadIdx.x + 192]));
    out[threadIdx.x] = acc[0] * 3.0f;
}
__global__ void probe_xdl_vgpr_read_padded(const f16x8* a, float* out) {
    pf32x16 acc;
    asm volatile("v_mfma_f32_32x32x16_f16 %0, %1, %2, 0" : "=&v"(acc) : "v"(a[threadIdx.x]), "v"(a[threadIdx.x + 64]));
    asm volatile("v_mfma_f32_32x32x16_f16 %0, %1, %2, %0\n\ts_nop 11" : "+v"(acc) : "v"(a[threadIdx.x + 128]), "v"(a[threadIdx.x + 192]));
    out[threadIdx.x] = acc[0] * 3.0f;
}

// VALU SGPR write -> asm VMEM read of it (the checker's fourth audit, round
// 6): a descriptor word fresh from v_readfirstlane read by an asm LDS-DMA
// opened with s_nop 0 only (the LDS-DMA helper's first "{m0}" form), and the
// same with the helper's s_nop 4
__device__ __forceinline__ i32x4 probe_srd(const uint8_t* p, const uint32_t* w) {
    i32x4 r;
    r.x = (int)(uint32_t)(uint64_t)p;
    r.y = (int)(uint32_t)((uint64_t)p >> 32);
    r.z = (int)__builtin_amdgcn_readfirstlane(w[threadIdx.x]);  // a loaded VGPR -> SGPR: a VALU write
    r.w = 0x00020000;
    return r;
}
__global__ void probe_sgpr_vmem(const uint8_t* p, const uint32_t* w, uint32_t lds) {
    const i32x4 srd = probe_srd(p, w);
    asm volatile("s_nop 0\n\tbuffer_load_dword %0, %1, 0 offen lds" : : "v"(threadIdx.x * 4), "s"(srd), "{m0}"(lds)
                 : "memory");
}
__global__ void probe_sgpr_vmem_padded(const uint8_t* p, const uint32_t* w, uint32_t lds) {
    const i32x4 srd = probe_srd(p, w);
    asm volatile("s_nop 4\n\tbuffer_load_dword %0, %1, 0 offen lds" : : "v"(threadIdx.x * 4), "s"(srd), "{m0}"(lds)
                 : "memory");
}
