"""Generate csrc/mel_tables.h: compile-time mel/DCT tables for the reference's
filterbank configurations, so mfcc_kernel's phase 2 compiles to straight-line
code (literal weights, immediate LDS offsets) instead of a scalar-load-driven
tap loop.

The tables are produced with the same arithmetic as the runtime plan
(vad_amd.mfcc.get_mel_filterbanks -> fp32 taps x 2^-20; lifter x DCT-II ortho
in fp64 -> fp32), and vad_mfcc_plan_create selects a specialised kernel only
when the runtime plan equals a table bit for bit.

    python -m vad_amd.gen_tables
"""
from __future__ import annotations

import math
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
OUT = os.path.join(HERE, "csrc", "mel_tables.h")
OUT_CODE = os.path.join(HERE, "csrc", "mel_code.h")

# (name, low_hz, high_hz, n_filters, sample_rate, mfcc_n, lifter)
CONFIGS = [
    ("Mel26", 300, 8000, 26, 16000, 13, 22),   # config.py:20-27, sklearn_analyser.py:21
    ("Mel40", 300, 8000, 40, 16000, 13, 22),   # BASELINE.json config 2
]
WAVES = 8          # phase-2a filter bands (one per wave) of mfcc_kernel
DCT_GROUPS = 4     # phase-2b coefficient groups c = g, g+4, ... (waves 0..3)


def mel_filterbank(lo, hi, nf, sr, fft_n=512):
    # identical arithmetic to vad_amd/mfcc.py::get_mel_filterbanks (mfcc.py:5-56)
    first_mel = 1125.0 * np.log(1.0 + lo / 700.0)
    last_mel = 1125.0 * np.log(1.0 + hi / 700.0)
    delta = (last_mel - first_mel) / (nf + 1)
    mels = [first_mel + i * delta for i in range(nf + 1)] + [last_mel]
    mels.sort()
    hz = [700 * (np.exp(m / 1125) - 1) for m in mels]
    b = np.asarray([np.floor((fft_n + 1) * h / sr) for h in hz], np.float64)
    k = np.arange(0, fft_n // 2, 1, dtype=np.float64)
    fb = np.zeros((nf, fft_n // 2))
    with np.errstate(divide="ignore", invalid="ignore"):
        for m in range(1, nf + 1):
            rise = (k >= b[m - 1]) & (k <= b[m])
            fall = (~rise) & (k >= b[m]) & (k <= b[m + 1])
            fb[m - 1, rise] = (k[rise] - b[m - 1] + 0.0) / (b[m] - b[m - 1] + 0.0)
            fb[m - 1, fall] = (b[m + 1] - k[fall] + 0.0) / (b[m + 1] - b[m] + 0.0)
    return fb


def dct_matrix(nf, nc, L):
    d = np.zeros((nc, nf))
    for c in range(nc):
        lift = 1.0 + (L / 2.0) * math.sin(math.pi * c / L) if L > 0 else 1.0
        sc = math.sqrt(1.0 / (4.0 * nf)) if c == 0 else math.sqrt(1.0 / (2.0 * nf))
        for m in range(nf):
            d[c, m] = lift * sc * 2.0 * math.cos(math.pi * c * (2.0 * m + 1.0) / (2.0 * nf))
    return d.astype(np.float32)


def bands(lens, waves):
    """Contiguous filter bands balanced by cost (taps + (==0 -> eps) + log10)."""
    nf = len(lens)
    cost = [lens[m] + 8 for m in range(nf)]
    total = sum(cost)
    band, acc, m = [0], 0, 0
    for w in range(waves):
        target = total * (w + 1) / waves
        while m < nf and (acc + cost[m] / 2 <= target or w == waves - 1):
            acc += cost[m]
            m += 1
        band.append(m)
    return band


def fhex(x):
    return float(np.float32(x)).hex() + "f"


def emit(name, lo, hi, nf, sr, nc, L):
    fb = mel_filterbank(lo, hi, nf, sr)
    assert np.isfinite(fb).all()
    los, lens, taps = [], [], []
    for m in range(nf):
        nz = np.nonzero(fb[m])[0]
        a, z = int(nz[0]), int(nz[-1])
        los.append(a)
        lens.append(z - a + 1)
        taps.append((fb[m, a:z + 1].astype(np.float32) * np.float32(2.0 ** -20)).astype(np.float32))
    dense = np.zeros((nf, 256), np.float32)
    for m in range(nf):
        dense[m, los[m]:los[m] + lens[m]] = taps[m]
    band = bands(lens, WAVES)
    d = dct_matrix(nf, nc, L)
    lines = [f"struct {name} {{",
             f"  static constexpr int NF = {nf};",
             f"  static constexpr int NC = {nc};",
             f"  static constexpr int lo[{nf}] = {{{', '.join(map(str, los))}}};",
             f"  static constexpr int len[{nf}] = {{{', '.join(map(str, lens))}}};",
             f"  static constexpr int band[{WAVES + 1}] = {{{', '.join(map(str, band))}}};",
             f"  // dense fp32 taps x 2^-20, [filter][bin]",
             f"  static constexpr float w[{nf}][256] = {{"]
    for m in range(nf):
        lines.append("    {" + ", ".join(fhex(v) if v != 0 else "0" for v in dense[m]) + "},")
    lines.append("  };")
    lines.append(f"  // lifter(L={L}) x DCT-II ortho, [coef][filter]")
    lines.append(f"  static constexpr float dct[{nc}][{nf}] = {{")
    for c in range(nc):
        lines.append("    {" + ", ".join(fhex(v) for v in d[c]) + "},")
    lines.append("  };")
    lines.append("};")
    return "\n".join(lines), (los, lens, taps, d, band, dense)


def bits(x):
    return "0x%08x" % int(np.float32(x).view(np.uint32))


def emit_code(name, info):
    """Straight-line phase-2 code: per wave band the mel energies and their
    log10 (mel_band_code), per coefficient group the lifter x DCT of a frame's
    log-mel row (dct_code).  One v_fmac_f32 with a 32-bit literal per tap /
    DCT term (VOP2 literal: no SGPR, nothing for the compiler to hoist out of
    the persistent tile loop and spill)."""
    los, lens, taps, d, band, dense = info
    out = mel_bands(name, los, lens, dense, band, WAVES, "mel_band_code")
    out += dct_groups(name, d, DCT_GROUPS, "dct_code")
    return "\n".join(out)


def mel_bands(name, los, lens, dense, band, waves, fname):
    out = []
    comp = "xyzw"
    for w in range(waves):
        fb, fe = band[w], band[w + 1]
        out.append(f"template <> __device__ __forceinline__ void {fname}<{name}, {w}>(")
        out.append("    const float* __restrict__ prow, float* __restrict__ lm) {")
        if fb == fe:
            out.append("  (void)prow;\n  (void)lm;\n}")
            continue
        k0 = los[fb] & ~3
        k1 = los[fe - 1] + lens[fe - 1]
        nq = (k1 - k0 + 3) // 4
        for q in range(nq):
            out.append(f"  const v4f q{q} = *reinterpret_cast<const v4f*>("
                       f"__builtin_assume_aligned(prow + {k0 + 4 * q}, 16));")
        # each filter's taps split into two interleaved sub-chains, all chains
        # of the band emitted round-robin (volatile: the order is the issue
        # order), so that no fmac consumes the accumulator written by the
        # instruction just before it -- more ILP and no hazard s_nops
        chains = []
        for m in range(fb, fe):
            tp = [(k, dense[m, k]) for k in range(k0, k1) if dense[m, k] != 0]
            halves = [tp[0::2], tp[1::2]] if len(tp) >= 4 else [tp]
            for h, t in enumerate(halves):
                chains.append((f"e{m - fb}_{h}", t))
        for reg, _ in chains:
            out.append(f"  float {reg};")
        for step in range(max(len(t) for _, t in chains)):
            for reg, t in chains:
                if step >= len(t):
                    continue
                k, v = t[step]
                q, r = divmod(k - k0, 4)
                src = f"q{q}.{comp[r]}"
                if step == 0:
                    out.append(f'  asm volatile("v_mul_f32_e32 %0, {bits(v)}, %1" : "=v"({reg}) : "v"({src}));')
                else:
                    out.append(f'  asm volatile("v_fmac_f32_e32 %0, {bits(v)}, %1" : "+v"({reg}) : "v"({src}));')
        for m in range(fb, fe):
            regs = [reg for reg, _ in chains if reg.startswith(f"e{m - fb}_")]
            out.append(f"  const float e{m - fb} = {' + '.join(regs)};")
        for m in range(fb, fe):
            out.append(f"  lm[{m}] = log10_pos(e{m - fb} == 0.f ? 0x1p-52f : e{m - fb});"
                       f"  // (==0 -> eps), log10")
        out.append("}")
        out.append("")
    return out


def dct_groups(name, d, ng, fname):
    """lifter x DCT of a log-mel row for the coefficient groups c = g + ng i
    (ng = 4: waves 0..3 own four coefficients each), one sequential fma chain
    per coefficient (the MFMA DCT's order)."""
    nf, nc = d.shape[1], d.shape[0]
    per = (nc + ng - 1) // ng
    comp = "xyzw"
    out = []
    nq = (nf + 3) // 4
    for g in range(ng):
        coefs = list(range(g, nc, ng))
        out.append(f"template <> __device__ __forceinline__ void {fname}<{name}, {g}>(")
        out.append(f"    const float* __restrict__ lm, float (&acc)[{per}]) {{")
        for q in range(nq):
            out.append(f"  const v4f q{q} = *reinterpret_cast<const v4f*>("
                       f"__builtin_assume_aligned(lm + {4 * q}, 16));")
        # one fma chain per coefficient, filters in ascending order from +0:
        # bit for bit the k-ordered chain of mfcc3_kernel's f32 MFMA DCT
        # (v_mfma_f32_16x16x4_f32), so every clip path gives the same MFCCs
        chains = []
        for i, c in enumerate(coefs):
            out.append(f"  float a{i} = 0.f;  // coefficient {c}")
            chains.append((f"a{i}", c))
        for m in range(nf):
            for reg, c in chains:
                q, r = divmod(m, 4)
                src = f"q{q}.{comp[r]}"
                out.append(f'  asm volatile("v_fmac_f32_e32 %0, {bits(d[c, m])}, %1" : "+v"({reg}) : "v"({src}));')
        for i in range(per):
            out.append(f"  acc[{i}] = a{i};" if i < len(coefs) else f"  acc[{i}] = 0.f;")
        out.append("}")
        out.append("")
    return out


def main():
    parts = ["// GENERATED by vad_amd/gen_tables.py -- do not edit.",
             "// Compile-time mel filterbank / lifter x DCT tables of the reference",
             "// configurations (mfcc.py:39-56, 72-93; config.py:20-27).",
             "#pragma once", "", "namespace vad {", ""]
    code = ["// GENERATED by vad_amd/gen_tables.py -- do not edit.",
            "// Straight-line phase-2 code for the compile-time filterbanks of",
            "// mel_tables.h: mel / log10 per wave band (phase 2a) and lifter x DCT",
            "// per coefficient group (phase 2b).  Included by mfcc_kernel.hip after",
            "// mel_band_code / dct_code / log10_pos are declared.",
            "#pragma once", ""]
    for cfg in CONFIGS:
        src, info = emit(*cfg)
        parts.append(src)
        parts.append("")
        code.append(emit_code(cfg[0], info))
    parts.append("}  // namespace vad")
    with open(OUT, "w") as f:
        f.write("\n".join(parts) + "\n")
    with open(OUT_CODE, "w") as f:
        f.write("\n".join(code) + "\n")
    print("wrote", OUT, OUT_CODE)


if __name__ == "__main__":
    main()
