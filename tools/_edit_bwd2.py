p = 'cuda-flash-attention_amd/kernels/f-attn2-backward_f16.cu'
s = open(p).read()


def rep(a, b, count=1):
    global s
    n = s.count(a)
    if n != count:
        raise SystemExit(f"pattern found {n}x (want {count}): {a[:90]!r}")
    s = s.replace(a, b)


i = s.index('// KB x 32 keys per wave, NW waves: grid BH * ceil(S / (32*KB*NK)), block 64*NW.')
j = s.index('// ---------------------------------------------------------------------------\n// dQ:  grid')
s = s[:i] + open('tools/_dkdv_body.txt').read() + '\n' + s[j:]

rep('''        if (NKB > 1 && kb == 1) mid();  // between the two key blocks (next tile's loads, FA2_DQ_LP)''',
    '''        if (NKB > 1 && kb == 1) mid();  // between the two key blocks (the next tile's loads)''')
rep('''        if (NKB > 1 && kb == 1) mid();  // the next tile's loads between the two 32-key halves (FA2_DQ_LP)''',
    '''        if (NKB > 1 && kb == 1) mid();  // the next tile's loads between the two 32-key halves''')
rep('// ---- dQ on v_mfma_f32_16x16x32 (FA2_TUNE_DQ_MF=16), maps as in dkdv_step16:',
    '// ---- dQ on v_mfma_f32_16x16x32, maps as in dkdv_step16:')
rep('    static constexpr int DBLK = OSTAGE + (FA2_BWD_COAL ? NQ * 32 * 36 * 4 : 0);',
    '    static constexpr int DBLK = OSTAGE + NQ * 32 * 36 * 4;')
rep('''#if FA2_BWD_COAL
    float(*ostage)[32][36] = reinterpret_cast<float(*)[32][36]>(lds + L::OSTAGE);  // per-wave dQ stage
#endif''', '''    float(*ostage)[32][36] = reinterpret_cast<float(*)[32][36]>(lds + L::OSTAGE);  // per-wave dQ stage''')
rep('''    static_assert(!M16 || FA2_BWD_COAL, "16x16x32 dQ: coalesced prologue");
''', '')
rep('''    // K/V staging by the first FA2_DQ_SW waves (all when 0), as in the dK/dV kernel
    constexpr int SW = (FA2_DQ_SW > 0 && FA2_DQ_SW < NW) ? FA2_DQ_SW : NW;''',
    '''    constexpr int SW = NW;  // K/V staging by every wave (by waves 0-3 only: no gain, r01)''')
rep('''    const int nsteps = (ntiles + KS - 1) / KS;
#if FA2_BWD_COAL
    // Prologue.  L::OVL''', '''    const int nsteps = (ntiles + KS - 1) / KS;
    // Prologue.  L::OVL''')
i = s.index('        if constexpr (!OVL) __syncthreads();\n    }\n#else\n#pragma unroll\n    for (int t = 0; t < D / 16; ++t) {\n        st.qf[t] = load_frag(Q')
j = s.index('#endif\n', i)
s = s[:i] + '        if constexpr (!OVL) __syncthreads();\n    }\n' + s[j + len('#endif\n'):]
rep('''#if FA2_BWD_COAL
        const float nd = !qvalid ? 0.f : DELTA ? -delta_blk[wave * 32 + r] : -Delta[(long)bh * S + q];
#else
        const float nd = qvalid ? -Delta[(long)bh * S + q] : 0.f;
#endif''', '''        const float nd = !qvalid ? 0.f : DELTA ? -delta_blk[wave * 32 + r] : -Delta[(long)bh * S + q];''')
rep('    if (FA2_DQ_PRIO && NW == 8 && __builtin_amdgcn_readfirstlane(tid >> 6) >= NW / 2) __builtin_amdgcn_s_setprio(1);',
    '    if (NW == 8 && __builtin_amdgcn_readfirstlane(tid >> 6) >= NW / 2) __builtin_amdgcn_s_setprio(1);')
rep('    if (!FA2_BWD_COAL || !L::OVL) {', '    if (!L::OVL) {')
rep('            if ((FA2_DQ_LOAD_ALWAYS || more) && !FA2_DQ_LP) ld();\n', '', 2)
rep('''            auto mid = [&] {
                if ((FA2_DQ_LOAD_ALWAYS || more) && FA2_DQ_LP) ld();
            };''', '''            auto mid = [&] { ld(); };  // also on the last step (see FA2_DKDV_SW's note)''', 2)
i = s.index('#if FA2_BWD_COAL\n    {\n        const int q0w = qb * 32 * NQ + wave * 32;')
j = s.index('#else\n    if (qvalid) {', i)
k = s.index('#endif\n', j)
s = s[:i] + s[i + len('#if FA2_BWD_COAL\n'):j] + s[k + len('#endif\n'):]
rep('''#ifndef FA2_STAMPS
// dK/dV and dQ in ONE launch (small grids).''', '''// dK/dV and dQ in ONE launch (small grids).''')
rep('''        dkdv_body<D, NW, 1, 0, true, QS>(lds, xcd_remap(b, ndk), b, Q, K, V, dO, LSE, Delta, dK, dV, S);''',
    '''        dkdv_body<D, NW, 1, true, QS>(lds, xcd_remap(b, ndk), Q, K, V, dO, LSE, Delta, dK, dV, S);''')
i = s.index('                                             const_cast<float*>(Delta), dQ, S, nullptr);\n}\n#endif\n')
s = s.replace('                                             const_cast<float*>(Delta), dQ, S, nullptr);\n}\n#endif\n',
              '                                             const_cast<float*>(Delta), dQ, S, nullptr);\n}\n', 1)
open(p, 'w').write(s)
print("stage2 ok")
