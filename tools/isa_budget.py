"""Per-phase VALU budget of the MFCC kernel from its ISA (verdict r05 item 2).

    python tools/isa_budget.py [--symbol SUBSTR] [--json OUT]

Compiles vad_amd/csrc/mfcc_kernel.hip with the library's flags plus line
tables (tools/isa.sh), takes the C3 instance (mfcc_kernel<float, 0, 13, true,
400, 1, 5, false>: fp32 clip, 26 mel, paired frames) and attributes every
instruction of its tile loop to a phase and an operation class:

  * phase 1 (FFT) is cut by the kernel's own milestone priorities
    (s_setprio 3 / 2 / 1 / 0, mfcc_kernel.hip VAD_MILESTONE): [3, 2) stage A
    of pass 0 + its transpose, [2, 1) stage A of pass 1, [1, 0) the finish
    (stage B DFT8s, real-FFT split, power) of pass 0, [0, end) pass 1's
    transpose and finish; inside a segment the innermost source line names
    the operation (fft_pk.h function, finish_b line);
  * phase 2a (mel + log10) is generated code (mel_code.h), one filter band
    per wave: every wave runs its own case, so a tile costs the SUM of the
    eight cases for 64 frames;
  * phase 2b (lifter x DCT, MFMA) runs on waves 0..3.

Per frame = wave-instructions per tile x waves running them / 64 frames
(phase 1 and the loop: 8 waves; phase 2b: 4).  Compare with the PMC count
(SQ_INSTS_VALU per frame, profiles/r05/val_r05l/pmc.txt: 89.46).
"""
from __future__ import annotations

import argparse
import collections
import json
import os
import re
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SYM = "_ZN3vad11mfcc_kernelIfLi0ELi13ELb1ELi400ELi1ELi5ELb0E"

# fft_pk.h line ranges -> operation (inline asm lines and expression lines)
FFT_PK = [((25, 32), "cmul"), ((33, 56), "add/sub (-i, conj)"), ((57, 69), "split_u/v"),
          ((70, 90), "const twiddle (mul_cs, w8_1)"), ((91, 112), "dft4 adds"), ((113, 127), "dft8 adds"),
          ((128, 160), "dft16 adds"), ((161, 182), "dft16 even/odd adds")]


def compile_isa(out):
    subprocess.run(["bash", os.path.join(REPO, "tools", "isa.sh"), "mfcc_kernel.hip", out, "-gline-tables-only"],
                   check=True, capture_output=True)


def parse(path, sym):
    files, lines, start = {}, open(path).read().split("\n"), None
    for i, l in enumerate(lines):
        m = re.match(r'\s*\.file\s+(\d+)\s+"[^"]*"\s+"([^"]+)"', l)
        if m:
            files[m.group(1)] = os.path.basename(m.group(2))
        if start is None and l.startswith(sym) and l.split(":")[0].startswith(sym):
            start = i
    if start is None:
        sys.exit(f"symbol {sym} not found")
    cur, out = ("?", 0), []
    for l in lines[start + 1:]:
        if l.startswith(".Lfunc_end"):
            break
        m = re.match(r"\s*\.loc\s+(\d+)\s+(\d+)", l)
        if m:
            cur = (files.get(m.group(1), m.group(1)), int(m.group(2)))
            continue
        m = re.match(r"^(\.LBB\w+):", l)
        if m:
            out.append(("LABEL", m.group(1), 0, ""))
            continue
        s = l.strip()
        if not s or s.startswith((";", ".")):
            continue
        out.append(("INSN", cur[0], cur[1], s))
    return out


def kind(ins):
    mn = ins.split()[0]
    if "mfma" in mn:
        return "mfma"
    if mn.startswith("v_pk_"):
        return "valu_packed"
    if mn.startswith("v_"):
        return "valu_scalar"
    if mn.startswith("ds_"):
        return "lds"
    if mn.startswith(("global_", "buffer_")):
        return "vmem"
    return "other"


def fft_op(line):
    for (a, b), name in FFT_PK:
        if a <= line <= b:
            return name
    return f"fft_pk.h:{line}"


def phase1_op(seg, f, ln):
    if f == "fft_pk.h":
        op = fft_op(ln)
        fin = seg.startswith(("1c", "1d"))
        if fin and op == "cmul":
            return "split twiddle W512^k (cmul)"
        if fin and op == "split_u/v":
            return "real-FFT split (U, V)"
        if fin and op == "add/sub (-i, conj)" and ln >= 45:
            return "real-FFT split (S, D)"
        if not fin and op == "cmul":
            return "stage-A twiddle W256 (cmul)"
        return op
    if f == "mfcc_kernel.hip":
        if 320 <= ln <= 322 or 330 <= ln <= 336:
            return "column-0 fix-ups (selects, bins 0/128)"
        if 327 <= ln <= 328:
            return "power |2X|^2"
        if 340 <= ln <= 358:
            return "power-row store addresses"
        if 253 <= ln <= 262:
            return "sample-load addresses"
        if 116 <= ln <= 126:
            return "zero padding"
        if 281 <= ln <= 302:
            return "transpose (store_a / read_b)"
        return "tile loop bookkeeping"
    return f"{f}:{ln}"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--symbol", default=SYM)
    ap.add_argument("--asm", default="/tmp/vad_isa_budget.s")
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    compile_isa(a.asm)
    ins = parse(a.asm, a.symbol)
    # the tile loop: from the block holding the first 's_setprio 3' to the
    # back edge that branches to that block
    i3 = next(i for i, x in enumerate(ins) if x[0] == "INSN" and x[3].startswith("s_setprio 3"))
    head = max(i for i in range(i3) if ins[i][0] == "LABEL")
    hlabel = ins[head][1]
    back = next(i for i in range(len(ins) - 1, head, -1)
                if ins[i][0] == "INSN" and re.search(r"s_c?branch\w*\s+" + re.escape(hlabel) + r"\b", ins[i][3]))
    body = ins[head:back + 1]
    # blocks of the loop: the header block is phase 1 (cut by the milestone
    # priorities); a block with an MFMA or dct_mfma16's lines (and the store
    # blocks right after it, up to the first barrier) is phase 2b; a block
    # with generated mel code is one wave's phase-2a case; the rest is loop
    # bookkeeping and the barriers, run by all eight waves
    blocks, cur = [], None
    for x in body:
        if x[0] == "LABEL":
            cur = [x[1], []]
            blocks.append(cur)
        else:
            cur[1].append(x[1:])
    seg = "loop head"
    rows = collections.defaultdict(collections.Counter)
    seen_barrier = False
    for bi, (label, insns) in enumerate(blocks):
        has_mel = any(f == "mel_code.h" for f, _, _ in insns)
        has_dct = any("mfma" in s_ or (f == "mfcc_kernel.hip" and 499 <= ln <= 520) for f, ln, s_ in insns)
        has_bar = any(s_.startswith("s_barrier") for _, _, s_ in insns)
        for f, ln, s in insns:
            k = kind(s)
            if bi == 0:
                m = re.match(r"s_setprio (\d)", s)
                if m:
                    seg = {"3": "1a stage A pass 0 + transpose", "2": "1b stage A pass 1",
                           "1": "1c finish pass 0", "0": "1d transpose + finish pass 1"}[m.group(1)]
                    continue
                rows[("phase 1", seg, phase1_op(seg, f, ln))][k] += 1
            elif has_mel:
                rows[("phase 2a", "mel + log10 (one case per wave)",
                      "mel taps" if f == "mel_code.h" else "log10 / eps select")][k] += 1
            elif has_dct or (not seen_barrier and not has_bar):
                rows[("phase 2b", "lifter x DCT (waves 0..3)", "MFMA DCT + MFCC stores")][k] += 1
            else:
                rows[("loop", "barriers, joins", f"{f}:{ln}" if f != "mfcc_kernel.hip" else "bookkeeping")][k] += 1
        seen_barrier = seen_barrier or has_bar
    # per-frame weights: phase 1 / loop code runs on 8 waves per 64-frame
    # tile, each mel case on one wave, the DCT on 4 waves
    def weight(ph, seg):
        return {"phase 2a": 1 / 64, "phase 2b": 4 / 64}.get(ph, 8 / 64)
    table, tot = [], collections.Counter()
    for (ph, seg, op), c in sorted(rows.items()):
        w = weight(ph, seg)
        r = {"phase": ph, "segment": seg, "op": op, "per_tile_wave": dict(c),
             "per_frame": {k: v * w for k, v in c.items()}}
        table.append(r)
        for k, v in c.items():
            tot[k] += v * w
    by_op = collections.defaultdict(collections.Counter)
    for r in table:
        for k, v in r["per_frame"].items():
            by_op[(r["phase"], r["op"] if r["phase"] == "phase 1" else r["segment"])][k] += v
    print(f"{'phase':9s} {'operation':46s} {'packed':>7s} {'scalar':>7s} {'mfma':>5s} {'lds':>5s}   (per frame)")
    for (ph, op), c in sorted(by_op.items(), key=lambda kv: (kv[0][0], -(kv[1]['valu_packed'] + kv[1]['valu_scalar']))):
        if c["valu_packed"] + c["valu_scalar"] + c["mfma"] + c["lds"] < 0.05:
            continue
        print(f"{ph:9s} {op[:46]:46s} {c['valu_packed']:7.2f} {c['valu_scalar']:7.2f} {c['mfma']:5.2f} {c['lds']:5.2f}")
    print(f"{'total':9s} {'':46s} {tot['valu_packed']:7.2f} {tot['valu_scalar']:7.2f} {tot['mfma']:5.2f} {tot['lds']:5.2f}"
          f"   VALU {tot['valu_packed'] + tot['valu_scalar'] + tot['mfma']:.2f} (PMC SQ_INSTS_VALU 89.46 incl. MFMA)")
    if a.json:
        with open(a.json, "w") as fo:
            json.dump({"symbol": a.symbol, "rows": table, "by_op": {f"{p} | {o}": dict(c) for (p, o), c in by_op.items()},
                       "total_per_frame": dict(tot)}, fo, indent=1)


if __name__ == "__main__":
    main()
