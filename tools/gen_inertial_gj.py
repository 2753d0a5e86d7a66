"""Generate orb_slam_fusion_amd/csrc/inertial_gj.inc: the fully unrolled
Gauss-Jordan solve of the n x n inertial system (n = 30: LastFrame, 15:
LastKeyFrame) on one wave with DPP64 row broadcasts.

Layout: lane li of each 16-lane row owns rows li (A) and li + 16 (B, n = 30
only) in the natural order; a row holds its n entries and b at index n.  A
pivot with |d| <= tiny (a zero or near-zero pivot, whose sign the natural
order could get wrong) is flagged: the caller then takes ldlt_wave (Eigen's
pivot order and semantics).  Pivot k reads row
k's entries from lane k % 16 of the lane's own row (v_fmac_f64_dpp
row_newbcast), so one instruction updates one entry; every row but the pivot
row takes -l_i times it (Gauss-Jordan: the rows above too, which costs nothing
extra in this layout), leaving D on the diagonal and D x in b.

Each asm block starts with s_nop 1 (a VALU write followed by a DPP read of the
same VGPR needs 2 wait states; a block's inputs may come straight from
compiler VALU code).  Within a block each entry's two FMAs read the pivot row's
register first through the row that does not write it.

    python tools/gen_inertial_gj.py > orb_slam_fusion_amd/csrc/inertial_gj.inc
"""
import sys

BLOCK = 7  # entries per asm block (2 FMAs each): 14 read-write operands + 2 multipliers + 1 immediate


def fmac(dst, src, mul):
    return f'"v_fmac_f64_dpp %{dst}, %{src}, -%{mul} row_newbcast:%[n] row_mask:0xf bank_mask:0xf\\n\\t"'


def block(n, k, js, rows):
    """asm statement updating entries js of the row halves in rows ("A", "B")
    for pivot k."""
    src_b = k >= 16
    ops, lines = [], []
    for j in js:
        i = len(ops)
        if rows == ("A", "B"):
            a, b = i, i + 1
            ops += [f'"+v"(rA[{j}])', f'"+v"(rB[{j}])']
            if not src_b:  # pivot row in A: B first reads A's register, then A updates in place
                lines += [fmac(b, a, "[lb]"), fmac(a, a, "[la]")]
            else:
                lines += [fmac(a, b, "[la]"), fmac(b, b, "[lb]")]
        else:
            # one half: the pivot row's register is in the updated half, or
            # read from the other half's register (not written here)
            h = rows[0]
            ops.append(f'"+v"(r{h}[{j}])')
            src_h = "B" if src_b else "A"
            if src_h == h:
                lines.append(fmac(i, i, f"[l{h.lower()}]"))
            else:
                ops_in = f"s{j}"
                lines.append(fmac(i, f"[{ops_in}]", f"[l{h.lower()}]"))
    ins = []
    if "A" in rows:
        ins.append('[la] "v"(lA)')
    if "B" in rows:
        ins.append('[lb] "v"(lB)')
    if len(rows) == 1 and ("B" if src_b else "A") != rows[0]:
        src = "rB" if src_b else "rA"
        ins += [f'[s{j}] "v"({src}[{j}])' for j in js]
    ins.append(f'[n] "i"({k % 16})')
    body = "\n".join(f"               {l}" for l in lines)
    return (f'  asm volatile("s_nop 1\\n\\t"\n{body}\n'
            f'               : {", ".join(ops)}\n               : {", ".join(ins)});\n')


def structure(n):
    """Entries of the assembled system that can be non-zero (assemble<MODE>,
    csrc/inertial_kernels.hip): the visual block (0..5), EdgeInertial's
    columns (current pose / velocity 0..8, the whole previous frame 15..29),
    the prior (15..29) -- one dense set -- and the random walks, which couple
    the current biases only to their own 3 x 3 block and the previous frame's
    same bias (9..11 <-> 24..26, 12..14 <-> 27..29)."""
    dense = set(range(9)) | (set(range(15, 30)) if n == 30 else set())
    groups = [dense, {9, 10, 11} | ({24, 25, 26} if n == 30 else set()),
              {12, 13, 14} | ({27, 28, 29} if n == 30 else set())]
    return {(i, j) for g in groups for i in g for j in g}


def gen(n):
    """Pivot k updates only the columns j > k where row k can be non-zero,
    and only the row halves holding a row i != k that can be non-zero in
    column k (the fill-in of every pivot is tracked): a skipped FMA would add
    -l * 0 or -0 * x, so the result is the dense elimination's."""
    two = n > 16
    nz = structure(n)
    out = [f"// ---- n = {n} ----------------------------------------------------------\n",
           f"template <>\n__device__ __forceinline__ int gj_pivots<{n}>(double (&rA)[{n + 1}], "
           f"double (&rB)[{n + 1}], int li, double& dA, double& dB, double tiny) {{\n",
           ]
    total = 0
    for k in range(n):
        src = "rB" if k >= 16 else "rA"
        out.append(f"  {{  // pivot {k}\n")
        out.append(f"    double d;\n    asm volatile(\"s_nop 1\\n\\tv_mov_b64_dpp %0, %1 row_newbcast:{k % 16} "
                   f"row_mask:0xf bank_mask:0xf\" : \"=v\"(d) : \"v\"({src}[{k}]));\n")
        # the select at the pivot itself (an empty asm pins it): sunk to the
        # solve's end it kept every pivot's d live
        if k < 16:
            out.append(f"    dA = li == {k} ? d : dA;\n    asm volatile(\"\" : \"+v\"(dA));\n")
        else:
            out.append(f"    dB = li == {k - 16} ? d : dB;\n    asm volatile(\"\" : \"+v\"(dB));\n")
        rows_k = [i for i in range(n) if i != k and (i, k) in nz]
        cols_k = [j for j in range(k + 1, n) if (k, j) in nz] + [n]
        for i in rows_k:
            for j in cols_k[:-1]:
                nz.add((i, j))
        halves = tuple(h for h, lo, hi in (("A", 0, 16), ("B", 16, 32)) if any(lo <= i < hi for i in rows_k))
        if halves:
            out.append("    double r = __builtin_amdgcn_rcp(d);\n    r = fma(r, fma(-d, r, 1.0), r);\n")
            if "A" in halves:
                out.append(f"    const double lA = li != {k} ? rA[{k}] * r : 0.0;\n")
            if "B" in halves:
                out.append(f"    const double lB = li + 16 != {k} ? rB[{k}] * r : 0.0;\n")
            per = BLOCK if len(halves) == 2 else 2 * BLOCK
            for s in range(0, len(cols_k), per):
                out.append(block(n, k, cols_k[s:s + per], halves))
            total += len(cols_k) * len(halves)
        out.append("  }\n")
    # the flags from the pivots each lane kept (lane li: pivots li, li + 16),
    # one ballot instead of compares at every pivot
    out.append(f"  // {total} FMAs (dense: {sum(n - k for k in range(n)) * (2 if two else 1)})\n"
               f"  // bit 0: a negative pivot, bit 1: a (near-)zero pivot (wave-uniform)\n"
               f"  const bool vA = li < {n}, vB = li + 16 < {n};\n"
               f"  const bool neg = (vA && dA < 0.0) || (vB && dB < 0.0);\n"
               f"  const bool small = (vA && fabs(dA) <= tiny) || (vB && fabs(dB) <= tiny);\n"
               f"  return (__ballot(neg) != 0 ? 1 : 0) | (__ballot(small) != 0 ? 2 : 0);\n}}\n\n")
    return "".join(out)


def main():
    sys.stdout.write("// Generated by tools/gen_inertial_gj.py -- do not edit.\n"
                     "// Gauss-Jordan pivots of the inertial system with DPP64 row broadcasts\n"
                     "// (see the generator's docstring); included by inertial_kernels.hip.\n"
                     "template <int n>\n__device__ int gj_pivots(double (&rA)[n + 1], double (&rB)[n + 1], "
                     "int li, double& dA, double& dB, double tiny);\n\n")
    for n in (30, 15):
        sys.stdout.write(gen(n))


if __name__ == "__main__":
    main()
