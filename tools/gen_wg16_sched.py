#!/usr/bin/env python3
"""Generate csrc/src/hip/wino_gemm16_sched.inc: the hand-scheduled K slice of the F(4x4,5x5) Conv2 GEMM
(wino_gemm16.hpp, production shape Cfg<1,4,96,2>: one transform point = 96 channels = 6 groups of 16 per
slice, two 16x16 MFMA blocks per wave sharing each B fragment, the 16-output fold of the previous point).

Why asm: the compiler's schedule of this slice (profiles/r06_conv2_sched/) runs each accumulator's MFMAs
as a dependent chain of 4 (40-cycle dependent latency against a 32-cycle issue), waits lgkmcnt(0) on the
group it just issued, and clusters the 128 fold FMAs into one VALU burst (SLP-packed v_pk_fma_f32). This
slice issues, per 16-channel group s:
  * the three ds_read_b128 of group s + 2 (two groups ahead, a 3-buffer fragment rotation, so a read
    never lands in a register an in-flight MFMA still reads as C, and group s + 1 is never waited for);
  * one counted wait, lgkmcnt(3) (group s only);
  * 8 MFMAs alternating the two blocks' accumulators (a dependent pair 64 cycles apart);
  * 2-3 fold FMAs behind every MFMA (v_fmac_f32, scalar coefficient; the same fmaf order as the C++ fold,
    so the output is bitwise identical to the compiler-scheduled kernel).
Fragment buffers are the literal registers v220-v255 (clobbered by the statement); everything else is
an operand. Reference op: convKernel (v3_cuda_only/src/layers_cuda.cu:20-46).

Run: python tools/gen_wg16_sched.py  (writes the .inc; the build does not run it).
"""
import os

G4 = 6        # 16-channel groups per slice (BK 96)
NQ, NE = 16, 8
FB = 220      # first fragment register: buffer b at v[FB + 12b ...]: A0 +0..3, A1 +4..7, B +8..11
NF = NQ * NE  # fold FMAs per point
MF = G4 * 8   # MFMAs per slice


def body(fold: bool, mode: int, pk: bool, dmode: int = 0):
    """mode: where the fold FMAs of the previous point go -- 0 behind every MFMA, 1 behind every group's 8
    MFMAs, 2 all at the slice start (under the first group's read latency), 3 half at the start, half
    behind the MFMAs. pk: v_pk_fma_f32 on filter-value pairs (the compiler's SLP form) instead of v_fmac_f32.
    dmode: the next point's LDS-DMA refill (3 V + 6 U pieces per wave) -- 0 not in the statement (issued by
    the caller, or none), 1 all at the statement start, 2 spread behind the MFMAs of groups 0-2, 3 behind the
    MFMAs of groups 0-4."""
    out = ["s_nop 4"] if dmode else []
    dmas = []
    for i in range(3):
        dmas.append([f"s_add_u32 m0, %[wb], %c[rs] + {i * 4096}", "s_nop 0",
                     f"buffer_load_dwordx4 %[voff{i}], %[vr], %[vso] offen lds"])
    for i in range(6):
        dmas.append([f"s_add_u32 m0, %[wb], %c[rs] + {12288 + i * 4096}", "s_nop 0",
                     f"buffer_load_dwordx4 %[uoff{i}], %[ur], %[uso] offen lds"])
    # dma slots: MFMA index after which each piece goes
    if dmode == 1:
        for d in dmas:
            out += d
        dslot = {}
    elif dmode == 2:
        dslot = {m: dmas[i] for i, m in enumerate([3, 5, 7, 11, 13, 15, 19, 21, 23])}
    elif dmode == 3:
        dslot = {m: dmas[i] for i, m in enumerate([3, 7, 11, 15, 19, 23, 27, 31, 35])}
    else:
        dslot = {}
    buf = lambda g: FB + 12 * (g % 3)
    def reads(g):
        b = buf(g)
        return [f"ds_read_b128 v[{b}:{b + 3}], %[ra0_{g}] offset:%c[so]",
                f"ds_read_b128 v[{b + 4}:{b + 7}], %[ra1_{g}] offset:%c[so]",
                f"ds_read_b128 v[{b + 8}:{b + 11}], %[rb_{g}] offset:%c[so]"]
    # the fold as a list of instructions in fmaf order (j = q * NE + e)
    fmas = []
    if fold:
        if pk:
            for q in range(NQ):
                sel = "op_sel_hi:[0,1,1]" if q % 2 == 0 else "op_sel:[1,0,0] op_sel_hi:[1,1,1]"
                for e2 in range(NE // 2):
                    fmas.append(f"v_pk_fma_f32 %[y{q}_{2 * e2}], %[c{q // 2}], %[p{e2}], %[y{q}_{2 * e2}] {sel}")
        else:
            for q in range(NQ):
                for e in range(NE):
                    fmas.append(f"v_fmac_f32 %[y{q}_{e}], %[c{q}], %[p{e}]")
    n = len(fmas)
    head = n // 2 if mode == 3 else (n if mode == 2 else 0)
    rest = fmas[head:]
    nr = len(rest)
    out += reads(0) + reads(1)
    out += fmas[:head]
    for s in range(G4):
        out.append(f"s_waitcnt lgkmcnt({3 if s + 1 < G4 else 0})")
        nxt = reads(s + 2) if s + 2 < G4 else []
        b = buf(s)
        for k in range(4):
            for blk in range(2):
                m = s * 8 + k * 2 + blk
                acc = f"%[a{blk}]"
                src_c = "0" if (s == 0 and k == 0) else acc
                out.append(f"v_mfma_f32_16x16x4_f32 {acc}, v{b + 4 * blk + k}, v{b + 8 + k}, {src_c}")
                i = k * 2 + blk
                if i < len(nxt):
                    out.append(nxt[i])
                if m in dslot:
                    out += dslot[m]
                if mode in (0, 3):
                    out += rest[nr * m // MF: nr * (m + 1) // MF]
        if mode == 1:
            out += rest[nr * s // G4: nr * (s + 1) // G4]
    return out


def func(fold: bool, mode: int = 0, pk: bool = False, dmode: int = 0):
    name = (f"slice_fold{mode}{'p' if pk else ''}" if fold else "slice_first") + f"_d{dmode}"
    sig = ["float (&Y)[16][8], f32x4& a0, f32x4& a1, const f32x4& p0, const f32x4& p1, const float (&c)[16],"
           if fold else "f32x4& a0, f32x4& a1,",
           "const int (&ra0)[6], const int (&ra1)[6], const int (&rb)[6]" +
           (", const Dma& d" if dmode else "")]
    outs = []
    pre = []
    if fold:
        if pk:
            outs += [f'[y{q}_{2 * e2}] "+v"(*reinterpret_cast<f32x2*>(&Y[{q}][{2 * e2}]))'
                     for q in range(NQ) for e2 in range(NE // 2)]
        else:
            outs += [f'[y{q}_{e}] "+v"(Y[{q}][{e}])' for q in range(NQ) for e in range(NE)]
    outs += ['[a0] "=&v"(a0)', '[a1] "=&v"(a1)']
    ins = []
    if fold:
        if pk:
            pre.append("  const f32x2 pp[4] = {f32x2{p0[0], p0[1]}, f32x2{p0[2], p0[3]}, f32x2{p1[0], p1[1]}, "
                       "f32x2{p1[2], p1[3]}};")
            pre.append("  f32x2 cc[8];")
            pre.append("#pragma unroll")
            pre.append("  for (int i = 0; i < 8; ++i) cc[i] = f32x2{c[2 * i], c[2 * i + 1]};")
            ins += [f'[p{e2}] "v"(pp[{e2}])' for e2 in range(NE // 2)]
            ins += [f'[c{i}] "s"(cc[{i}])' for i in range(NQ // 2)]
        else:
            ins += [f'[p{e}] "v"(p{e >> 2}[{e & 3}])' for e in range(NE)]
            ins += [f'[c{q}] "s"(c[{q}])' for q in range(NQ)]
    for g in range(G4):
        ins += [f'[ra0_{g}] "v"(ra0[{g}])', f'[ra1_{g}] "v"(ra1[{g}])', f'[rb_{g}] "v"(rb[{g}])']
    ins.append('[so] "i"(SO)')
    if dmode:
        ins += [f'[voff{i}] "v"(d.voff[{i}])' for i in range(3)] + [f'[uoff{i}] "v"(d.uoff[{i}])' for i in range(6)]
        ins += ['[vr] "s"(d.vr)', '[ur] "s"(d.ur)', '[vso] "s"(d.vso)', '[uso] "s"(d.uso)', '[wb] "s"(d.wb)',
                '[rs] "i"(RS)']
    clob = [f'"v{r}"' for r in range(FB, FB + 36)] + ['"memory"']
    lines = [f"template <int SO, int RS = 0>", f"__device__ __forceinline__ void {name}(" + sig[0], "    " + sig[1] + ") {"]
    lines += pre
    lines.append("  asm volatile(")
    lines += [f'      "{ins_}\\n\\t"' for ins_ in body(fold, mode, pk, dmode)]
    lines.append("      : " + ",\n        ".join(outs))
    lines.append("      : " + ",\n        ".join(ins))
    lines.append("      : " + ", ".join(clob) + ");")
    lines.append("}")
    return "\n".join(lines)


def main():
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    path = os.path.join(root, "csrc", "src", "hip", "wino_gemm16_sched.inc")
    text = ["// GENERATED by tools/gen_wg16_sched.py -- do not edit. The hand-scheduled K slice of the",
            "// F(4x4,5x5) Conv2 GEMM (wino_gemm16.hpp, ABL bit 64 / knob conv2_sched): see the generator's docstring.",
            "// Included inside namespace anx::hip::wg16 (f32x4 from wino_gemm.hpp).",
            "#pragma once", "", "typedef float f32x2 __attribute__((ext_vector_type(2)));", "",
            "// the next point's LDS-DMA refill: per-lane source offsets, buffer resources, per-point source",
            "// offsets and this wave's LDS byte base (wave * 1 KiB); RS (template) is the refill slot's byte offset",
            "struct Dma {", "  int voff[3], uoff[6];", "  __amdgpu_buffer_rsrc_t vr, ur;", "  int vso, uso, wb;", "};", ""]
    for dmode in range(4):
        text += [func(False, 0, False, dmode), ""]
    for mode, pk in ((0, False), (1, True), (2, True)):
        for dmode in range(4):
            text += [func(True, mode, pk, dmode), ""]
    with open(path, "w") as f:
        f.write("\n".join(text))
    print("wrote", path)


if __name__ == "__main__":
    main()
