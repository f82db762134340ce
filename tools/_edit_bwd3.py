p = 'cuda-flash-attention_amd/kernels/f-attn2-backward_f16.cu'
s = open(p).read()


def rep(a, b, count=1):
    global s
    n = s.count(a)
    if n != count:
        raise SystemExit(f"pattern found {n}x (want {count}): {a[:90]!r}")
    s = s.replace(a, b)


i = s.index('namespace {\n#ifdef FA2_STAMPS\nstruct StampLog')
j = s.index('template <int D, int NW, int NKB = 2, bool M16 = false, int KS = 1>\nhipError_t dq_launch')
s = s[:i] + r'''namespace {
// dK/dV kernel instances (NW waves x 32 keys; QS query groups).  16x16x32 everywhere
// but the 2-wave instance: at the power cap on random data 16x16x32 delivers 16 %
// more FLOPs per joule than 32x32x16 (+5 % at C3, +4 % at D = 128, +7 % on small
// D = 64 grids); the 2-wave instance keeps 32x32x16.
template <int D, int NW, bool M16 = true, int QS = 1>
hipError_t dkdv_launch(const float* q, const float* k, const float* v, const float* dout, const float* lse,
                       const float* delta, float* dk, float* dv, int bh, int S, hipStream_t stream) {
    const long grid = (long)bh * ((S + 32 * (NW / QS) - 1) / (32 * (NW / QS)));
    if (grid <= 0 || grid > 0x7fffffffL) return hipErrorInvalidValue;
    hipLaunchKernelGGL((fa2f16b::fa2_bwd_dkdv_f16_kernel<D, NW, 1, M16, QS>), dim3((unsigned)grid), dim3(64 * NW), 0,
                       stream, q, k, v, dout, lse, delta, dk, dv, S);
    return hipGetLastError();
}
// Geometry: 8 waves x 32 keys for D <= 64 (2 waves/SIMD in 256 VGPRs); D = 128 4 x 32
// (more than 256 registers per lane); fewer waves where the grid would leave CUs idle.
// Launch-plan overrides (fa2_tune_set, tests and tools only): DKDV_WAVES, DKDV_QS.
template <int D>
hipError_t dkdv_dispatch(const float* q, const float* k, const float* v, const float* dout, const float* lse,
                         const float* delta, float* dk, float* dv, int bh, int S, hipStream_t stream) {
    int nw = tune_knob("DKDV_WAVES", 0);  // 0 = auto_waves over the grid of 32-key wave units
    const long units = (long)bh * ((S + 31) / 32);
    // Query groups per workgroup (0 = auto).  Auto, where 8-wave workgroups of one key
    // block per wave would leave CUs idle: below 8 key blocks per CU QS = 2 at 8 waves;
    // below 4, D = 32 QS = 4 at 8 waves and D = 64 QS = 2 at 4 waves (at QS = 4 its
    // 4-tile staging registers spill).  Measured (B2_H8_D64, r01): S = 512 16.1 -> 12.1
    // us, 1024 29.1 -> 20.8, 2048 53.7 -> 44.3.
    int qs = tune_knob("DKDV_QS", 0);
    if (qs == 0 && nw == 0 && D <= 64) {
        const int a = auto_waves(units, 8);
        if (a == 4) qs = 2, nw = 8;
        else if (a == 2 && D <= 32) qs = 4, nw = 8;
        else if (a == 2) qs = 2, nw = 4;
    }
    if (nw == 0) nw = auto_waves(units, D <= 64 ? 8 : 4);
    if constexpr (D <= 64) {
        if (qs == 2 && nw == 8) return dkdv_launch<D, 8, true, 2>(q, k, v, dout, lse, delta, dk, dv, bh, S, stream);
        if (qs == 2 && nw == 4) return dkdv_launch<D, 4, true, 2>(q, k, v, dout, lse, delta, dk, dv, bh, S, stream);
        if (nw == 8) return dkdv_launch<D, 8>(q, k, v, dout, lse, delta, dk, dv, bh, S, stream);
    }
    if constexpr (D <= 32) {
        if (qs == 4 && nw == 8) return dkdv_launch<D, 8, true, 4>(q, k, v, dout, lse, delta, dk, dv, bh, S, stream);
    }
    if (nw == 2) return dkdv_launch<D, 2, false>(q, k, v, dout, lse, delta, dk, dv, bh, S, stream);
    return dkdv_launch<D, 4>(q, k, v, dout, lse, delta, dk, dv, bh, S, stream);
}
''' + s[j:]
rep('''#if FA2_BWD_COAL
    if (o)
        hipLaunchKernelGGL((fa2f16b::fa2_bwd_dq_f16_kernel<D, NW, true, NKB, M16, KS>), dim3((unsigned)grid),
                           dim3(64 * NW), 0, stream, q, k, v, dout, lse, delta, dq, S, o);
    else
#endif
''', '''    if (o)
        hipLaunchKernelGGL((fa2f16b::fa2_bwd_dq_f16_kernel<D, NW, true, NKB, M16, KS>), dim3((unsigned)grid),
                           dim3(64 * NW), 0, stream, q, k, v, dout, lse, delta, dq, S, o);
    else
''')
rep('''    // 8 waves (2 per SIMD) for D <= 64; at D = 128 8 waves spill (~120 VGPRs), so 4
    // FA2_TUNE_DQ_WAVES = 0 (default): auto_waves over the grid of 32-query wave units
    int nw = tune_knob("DQ_WAVES", 0);''', '''    // 8 waves (2 per SIMD) for D <= 64; at D = 128 8 waves spill (~120 VGPRs), so 4.
    // Launch-plan overrides (fa2_tune_set, tests and tools only): DQ_WAVES, DQ_KS.
    int nw = tune_knob("DQ_WAVES", 0);  // 0 = auto_waves over the grid of 32-query wave units''')
rep('''    // FA2_TUNE_DQ_KS: key groups per workgroup (0 = auto).''', '''    // Key groups per workgroup (0 = auto).''')
i = s.index('    // FA2_TUNE_DQ_MF: MFMA shape, 16 (16x16x32, default: +2.4 % at C3) or 32 (32x32x16)')
j = s.index('}\n', s.index('    return dq_launch<D, 4>(q, k, v, dout, lse, delta, dq, bh, S, o, stream);', i))
s = s[:i] + '''    // 16x16x32 (+2.4 % at C3 over 32x32x16) but at 2 waves
    if constexpr (D <= 64) {
        if (nw == 8) return dq_launch<D, 8, 2, true>(q, k, v, dout, lse, delta, dq, bh, S, o, stream);
        if (nw == 2) return dq_launch<D, 2>(q, k, v, dout, lse, delta, dq, bh, S, o, stream);
    }
    return dq_launch<D, 4, 2, true>(q, k, v, dout, lse, delta, dq, bh, S, o, stream);
''' + s[j:]
rep('''namespace {
#ifndef FA2_STAMPS
template <int D, int NW, int QS, int KS, int NKB>
hipError_t fused_launch(''', '''namespace {
template <int D, int NW, int QS, int KS, int NKB>
hipError_t fused_launch(''')
rep('''    return hipGetLastError();
}
#endif
// The fused dK/dV + dQ launch''', '''    return hipGetLastError();
}
// The fused dK/dV + dQ launch''')
rep('''// KS = 2, else unsplit.  FA2_TUNE_BWD_FQS / FA2_TUNE_BWD_FKS force them.''',
    '''// KS = 2, else unsplit.  Overrides (fa2_tune_set): BWD_FQS, BWD_FKS, BWD_FNW.''')
rep('''                          const float* delta, float* dq, float* dk, float* dv, int bh, int S, hipStream_t stream) {
#ifdef FA2_STAMPS
    return hipErrorNotSupported;
#else
    if constexpr (D > 64) {''', '''                          const float* delta, float* dq, float* dk, float* dv, int bh, int S, hipStream_t stream) {
    if constexpr (D > 64) {''')
rep('''        // FA2_TUNE_BWD_FNW: waves per workgroup of both roles (8, or 4 for the split pairs)''',
    '''        // waves per workgroup of both roles (8, or 4 for the split pairs)''')
rep('''        return hipErrorNotSupported;
    }
#endif
}''', '''        return hipErrorNotSupported;
    }
}''')
rep('''// FA2_TUNE_BWD_FUSED: 1 = Δ kernel, then dK/dV and dQ in one launch (D <= 64);''',
    '''// Override BWD_FUSED (fa2_tune_set): 1 = Δ kernel, then dK/dV and dQ in one launch (D <= 64);''')
open(p, 'w').write(s)
print("stage3 ok")
