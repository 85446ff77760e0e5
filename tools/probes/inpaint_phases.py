"""Diagnostic copy of csrc/dsx_inpaint.hip with per-evaluation phase stamps: with DSX_INPAINT_STAMPS set,
every step line also carries one evaluating group's entry time (us after the step's start) and its four
phases (row loads + staging, centre + terms, the fold, the stores and tags).  Build and run:
    python tools/probes/inpaint_phases.py depthestimation_amd/csrc/dsx_inpaint.hip /tmp/vp/dsx_inpaint.hip
    SRC=/tmp/vp/dsx_inpaint.hip OUTDIR=tools/varlib bash tools/variant_tu.sh phases dsx_inpaint
    DSX_LIB=$GRAFT_REPO_ROOT/tools/varlib/libdsx_phases.so bash tools/gpu_inpaint.sh stamps   (GPU box)
"""
import sys
src, dst = sys.argv[1], sys.argv[2]
s=open(src).read()
def rep(a,b,cnt=1):
    global s
    assert s.count(a)==cnt,(a[:60],s.count(a))
    s=s.replace(a,b)
rep("    double bound;\n};\n","    double bound;\n    unsigned long long *ph;\n};\n")
rep("    const Mode m = decide<RW>(S, mcv, __ballot(tg != 0u) != 0ull);\n",
    "    Mode m = decide<RW>(S, mcv, __ballot(tg != 0u) != 0ull);\n    m.ph = a.stamps && s < a.nstamps ? a.stamps + 8 * (size_t)s : nullptr;\n")
rep("    constexpr int NC = WN::NC, R = WN::R, ND = WN::ND, GL = WN::GL;\n    const int j = (int)(threadIdx.x & (GL - 1));\n",
    "    constexpr int NC = WN::NC, R = WN::R, ND = WN::ND, GL = WN::GL;\n    const int j = (int)(threadIdx.x & (GL - 1));\n    const unsigned long long ph0 = __builtin_amdgcn_s_memrealtime();\n    unsigned long long ph1 = 0, ph2 = 0, ph3 = 0;\n    auto phw = [&]() {\n        if (m.ph && j == 0) {\n            const unsigned long long t4 = __builtin_amdgcn_s_memrealtime();\n            auto c16 = [](unsigned long long d) { return d > 65535ull ? 65535ull : d; };\n            m.ph[5] = c16(ph1 - ph0) | c16(ph2 - ph1) << 16 | c16(ph3 - ph2) << 32 | c16(t4 - ph3) << 48;\n            m.ph[6] = ph0;\n        }\n    };\n")
rep("    if (rowv) L.av[j] = (uint16_t)avail;\n    wave_lds_sync();\n","    if (rowv) L.av[j] = (uint16_t)avail;\n    ph1 = __builtin_amdgcn_s_memrealtime();\n    wave_lds_sync();\n")
rep("    }\n    wave_lds_sync();\n    // OpenCV's sums","    }\n    ph2 = __builtin_amdgcn_s_memrealtime();\n    wave_lds_sync();\n    // OpenCV's sums")
rep("    wave_lds_sync();  // the group's LDS is reused by its next child\n    tc = tp;\n","    wave_lds_sync();  // the group's LDS is reused by its next child\n    ph3 = __builtin_amdgcn_s_memrealtime();\n    tc = tp;\n")
rep("    if (!changed) return;\n    if (j == 0) {\n        a.T[c] = tp;\n        a.out[c] = v;\n    }\n    if (sweep == 0) return;",
    "    if (!changed) { phw(); return; }\n    if (j == 0) {\n        a.T[c] = tp;\n        a.out[c] = v;\n    }\n    if (sweep == 0) { phw(); return; }")
rep("    for (int o = 1; o < GL; o <<= 1) dany |= __shfl_xor(dany, o, GL);\n    tagged = tagged || dany;\n}\n",
    "    for (int o = 1; o < GL; o <<= 1) dany |= __shfl_xor(dany, o, GL);\n    tagged = tagged || dany;\n    phw();\n}\n")
rep('''                            (unsigned)r[3], (unsigned)(r[3] >> 32), b0);''',
'''                            (unsigned)r[3], (unsigned)(r[3] >> 32), b0);
                    if (r[6]) fprintf(f, " entry %.2f ph %.2f %.2f %.2f %.2f", (double)((long long)(r[6] - r[0])) / 100.0,
                                      (double)(r[5] & 0xFFFF) / 100.0, (double)((r[5] >> 16) & 0xFFFF) / 100.0,
                                      (double)((r[5] >> 32) & 0xFFFF) / 100.0, (double)(r[5] >> 48) / 100.0);''')
rep('''                    fprintf(f, "%u %.2f %u %u %u %u %u %u %u %.2f\\n", i''','''                    fprintf(f, "%u %.2f %u %u %u %u %u %u %u %.2f", i''')
rep('''                }
                fprintf(f, "end\\n");''','''                    fprintf(f, "\\n");
                }
                fprintf(f, "end\\n");''')
open(dst,'w').write(s)
