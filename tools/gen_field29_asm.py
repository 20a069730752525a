"""Generate ntt_amd/csrc/field29_asm9.hpp: the L = 9 (256-bit class) radix-2^29 products with one
inline-asm statement per product column.

Why: gfx950's hazard recognizer separates two DEPENDENT inline-asm VALU statements with an s_nop
(it assumes a DST_SEL forwarding hazard it cannot rule out inside asm), and an s_nop costs a full
4-cycle issue slot.  One statement per column puts a compiler-generated instruction (the column's
shift / mask) between any two statements, so no pads are inserted, and keeps every column a single
dependent v_mad_u64_u32 chain (no second chain re-joined by a 64-bit add, which the compiler
builds for the plain C++ form).

    python tools/gen_field29_asm.py > ntt_amd/csrc/field29_asm9.hpp
"""
import sys
L = 9


def mads(pairs, first_idx):
    """asm body + operand list for acc += sum a*b over pairs [(a_expr, b_expr, b_is_sgpr)]."""
    lines, ops = [], []
    k = first_idx
    for a, b, bs in pairs:
        lines.append(f"v_mad_u64_u32 %0, %1, %{k}, %{k + 1}, %0")
        ops.append(f'"v"({a})')
        ops.append(f'"{"s" if bs else "v"}"({b})')
        k += 2
    return lines, ops


def stmt(pairs, indent="  "):
    lines, ops = mads(pairs, 2)
    body = "\\n\\t".join(lines)
    out = [f'{indent}asm("{body}"', f'{indent}    : "+v"(acc), "=&s"(cc)']
    # wrap operands 6 per line
    oplines = [", ".join(ops[i:i + 6]) for i in range(0, len(ops), 6)]
    out.append(f"{indent}    : " + (",\n" + indent + "      ").join(oplines) + ");")
    return "\n".join(out)


def gen_mulc(uniform=False):
    """uniform: the twiddle (w, ws) is wave-uniform (the w_8 / w_4 constants): SGPR operands, so the
    compiler does not copy its 18 words into VGPRs before every product."""
    o = []
    name = "mulc29_a9u" if uniform else "mulc29_a9"
    o.append(f"__device__ __forceinline__ void {name}(uint32_t (&r)[9], const uint32_t (&x)[9], const uint32_t (&w)[9],")
    o.append("                                          const uint32_t (&ws)[9], const uint32_t (&pbar)[9]) {")
    o.append("  uint32_t q[9];")
    o.append("  uint64_t acc = 0, cc;")
    o.append("  // q = floor(x * ws / B) from columns >= 7 (see mulc29)")
    for K in range(L - 2, 2 * L - 1):
        lo, hi = max(0, K - (L - 1)), min(K, L - 1)
        pairs = [(f"x[{i}]", f"ws[{K - i}]", uniform) for i in range(lo, hi + 1)]
        o.append(stmt(pairs))
        if K >= L:
            o.append(f"  q[{K - L}] = (uint32_t)acc & kMask29;")
        o.append("  acc >>= 29;")
    o.append("  q[8] = (uint32_t)acc;")
    o.append("  acc = 0;")
    o.append("  // r = (x * w + q * pbar) mod B")
    for K in range(L):
        pairs = [(f"x[{i}]", f"w[{K - i}]", uniform) for i in range(K + 1)]
        pairs += [(f"q[{i}]", f"pbar[{K - i}]", True) for i in range(K + 1)]
        o.append(stmt(pairs))
        o.append(f"  r[{K}] = (uint32_t)acc & kMask29;")
        if K + 1 < L:
            o.append("  acc >>= 29;")
    o.append("}")
    return "\n".join(o)


def gen_mont():
    o = []
    o.append("__device__ __forceinline__ void mont29_a9(uint32_t (&r)[9], const uint32_t (&a)[9], const uint32_t (&b)[9],")
    o.append("                                          const Mod29<9>& M) {")
    o.append("  uint32_t m[9];")
    o.append("  uint64_t acc = 0, cc;")
    for i in range(L):
        pairs = [(f"a[{j}]", f"b[{i - j}]", False) for j in range(i + 1)]
        pairs += [(f"m[{j}]", f"M.p[{i - j}]", True) for j in range(i)]
        o.append(stmt(pairs))
        o.append(f"  m[{i}] = ((uint32_t)acc * M.pinv) & kMask29;")
        o.append(stmt([(f"m[{i}]", "M.p[0]", True)]))
        o.append("  acc >>= 29;")
    for i in range(L, 2 * L):
        pairs = [(f"a[{j}]", f"b[{i - j}]", False) for j in range(i - L + 1, L)]
        pairs += [(f"m[{j}]", f"M.p[{i - j}]", True) for j in range(i - L + 1, L)]
        if pairs:
            o.append(stmt(pairs))
        o.append(f"  r[{i - L}] = (uint32_t)acc & kMask29;")
        if i + 1 < 2 * L:
            o.append("  acc >>= 29;")
    o.append("}")
    return "\n".join(o)


# ---------------------------------------------------------------- paired columns
# The column form above is ONE dependent v_mad_u64_u32 chain per product: 93 % of the MADs of the
# radix-256 column pass read the accumulator the previous instruction wrote (tools/isa_chains.py),
# and products run back to back, so a wave's MADs never overlap.  Here two adjacent columns K and
# K + 1 share one asm statement as two chains whose MADs alternate: column K + 1 starts from 0
# instead of from column K's carry, and the carry is added after both (one 64-bit add per column
# pair).  The sums are the same values as the single chain's (same bounds), with 2 more VGPRs.
def stmt2(pa, pb, indent="  "):
    """one statement: chain A (acc, carried in) and chain B (accb, from 0) with alternating MADs."""
    lines, ops = [], []
    k = 4
    ia = ib = 0
    first_b = True
    while ia < len(pa) or ib < len(pb):
        for which in ("a", "b"):
            if which == "a" and ia < len(pa):
                a, b, bs = pa[ia]
                ia += 1
                lines.append(f"v_mad_u64_u32 %0, %2, %{k}, %{k + 1}, %0")
            elif which == "b" and ib < len(pb):
                a, b, bs = pb[ib]
                ib += 1
                lines.append(f"v_mad_u64_u32 %1, %3, %{k}, %{k + 1}, {'0' if first_b else '%1'}")
                first_b = False
            else:
                continue
            ops.append(f'"v"({a})')
            ops.append(f'"{"s" if bs else "v"}"({b})')
            k += 2
    body = "\\n\\t".join(lines)
    out = [f'{indent}asm("{body}"', f'{indent}    : "+v"(acc), "=&v"(accb), "=&s"(cc), "=&s"(cc2)']
    oplines = [", ".join(ops[i:i + 6]) for i in range(0, len(ops), 6)]
    out.append(f"{indent}    : " + (",\n" + indent + "      ").join(oplines) + ");")
    return "\n".join(out)


def gen_mulc_pair(uniform=False):
    o = []
    name = "mulc29_a9u" if uniform else "mulc29_a9"
    o.append(f"__device__ __forceinline__ void {name}(uint32_t (&r)[9], const uint32_t (&x)[9], const uint32_t (&w)[9],")
    o.append("                                          const uint32_t (&ws)[9], const uint32_t (&pbar)[9]) {")
    o.append("  uint32_t q[9];")
    o.append("  uint64_t acc = 0, accb, cc, cc2;")
    o.append("  // q = floor(x * ws / B) from columns >= 7 (see mulc29), columns in pairs (7, 8) ... (15, 16)")
    cols = list(range(L - 2, 2 * L - 1))
    hi_terms = lambda K: [(f"x[{i}]", f"ws[{K - i}]", uniform) for i in range(max(0, K - (L - 1)), min(K, L - 1) + 1)]
    for a in range(0, len(cols), 2):
        K = cols[a]
        if a + 1 < len(cols):
            o.append(stmt2(hi_terms(K), hi_terms(K + 1)))
            if K >= L:
                o.append(f"  q[{K - L}] = (uint32_t)acc & kMask29;")
            o.append("  accb += acc >> 29;")
            if K + 1 >= L:
                o.append(f"  q[{K + 1 - L}] = (uint32_t)accb & kMask29;")
            o.append("  acc = accb >> 29;")
        else:
            o.append(stmt(hi_terms(K)))
            if K >= L:
                o.append(f"  q[{K - L}] = (uint32_t)acc & kMask29;")
            o.append("  acc >>= 29;")
    o.append("  q[8] = (uint32_t)acc;")
    o.append("  acc = 0;")
    o.append("  // r = (x * w + q * pbar) mod B, columns in pairs (0, 1) ... (6, 7), then 8")
    lo_terms = lambda K: ([(f"x[{i}]", f"w[{K - i}]", uniform) for i in range(K + 1)] +
                          [(f"q[{i}]", f"pbar[{K - i}]", True) for i in range(K + 1)])
    for K in range(0, L, 2):
        if K + 1 < L:
            o.append(stmt2(lo_terms(K), lo_terms(K + 1)))
            o.append(f"  r[{K}] = (uint32_t)acc & kMask29;")
            o.append("  accb += acc >> 29;")
            o.append(f"  r[{K + 1}] = (uint32_t)accb & kMask29;")
            if K + 2 < L:
                o.append("  acc = accb >> 29;")
        else:
            o.append(stmt(lo_terms(K)))
            o.append(f"  r[{K}] = (uint32_t)acc & kMask29;")
    o.append("}")
    return "\n".join(o)


# ---------------------------------------------------------------- one asm statement per product
# The column form above still pays hipcc's fixed boundary pad (an s_nop after every ;;#ASMEND whose
# outputs a VALU reads next): ~17 per product.  Here the whole product, shifts and masks included, is
# one statement, so the pad is paid once per product.  The 64-bit accumulator is the clobbered pair
# v[ACC:ACC+1] (inline asm cannot name the low half of a 64-bit operand).  No wait states are
# needed inside: every dependency is an ordinary VALU -> VALU one (no DPP / SDWA / op_sel / trans).
ACC = 126
MASK = "0x1fffffff"


def _whole(lines, outs, ins, clobbers, indent="  "):
    body = "\\n\\t".join(lines)
    o = [f'{indent}asm("{body}"']
    o.append(f"{indent}    : " + ", ".join(outs))
    o.append(f"{indent}    : " + (",\n" + indent + "      ").join(", ".join(ins[i:i + 6]) for i in range(0, len(ins), 6)))
    o.append(f"{indent}    : " + ", ".join(f'"{c}"' for c in clobbers) + ");")
    return "\n".join(o)


def gen_mulc_whole():
    A = f"v[{ACC}:{ACC + 1}]"
    R, Qo, CC, X, W, WS, PB = 0, L, 2 * L, 2 * L + 1, 3 * L + 1, 4 * L + 1, 5 * L + 1
    lines = []
    first = True
    for K in range(L - 2, 2 * L - 1):  # q = floor(x * ws / B) from columns >= L-2
        for i in range(max(0, K - (L - 1)), min(K, L - 1) + 1):
            lines.append(f"v_mad_u64_u32 {A}, %{CC}, %{X + i}, %{WS + K - i}, {'0' if first else A}")
            first = False
        if K >= L:
            lines.append(f"v_and_b32 %{Qo + K - L}, {MASK}, v{ACC}")
        lines.append(f"v_lshrrev_b64 {A}, 29, {A}")
    lines.append(f"v_mov_b32 %{Qo + L - 1}, v{ACC}")
    for K in range(L):  # r = (x * w + q * pbar) mod B
        for i in range(K + 1):
            lines.append(f"v_mad_u64_u32 {A}, %{CC}, %{X + i}, %{W + K - i}, {'0' if K == 0 and i == 0 else A}")
        for i in range(K + 1):
            lines.append(f"v_mad_u64_u32 {A}, %{CC}, %{Qo + i}, %{PB + K - i}, {A}")
        lines.append(f"v_and_b32 %{R + K}, {MASK}, v{ACC}")
        if K + 1 < L:
            lines.append(f"v_lshrrev_b64 {A}, 29, {A}")
    outs = [f'"=&v"(r[{k}])' for k in range(L)] + [f'"=&v"(q[{k}])' for k in range(L)] + ['"=&s"(cc)']
    ins = ([f'"v"(x[{k}])' for k in range(L)] + [f'"v"(w[{k}])' for k in range(L)] +
           [f'"v"(ws[{k}])' for k in range(L)] + [f'"s"(pbar[{k}])' for k in range(L)])
    o = ["__device__ __forceinline__ void mulc29_a9(uint32_t (&r)[9], const uint32_t (&x)[9], const uint32_t (&w)[9],",
         "                                          const uint32_t (&ws)[9], const uint32_t (&pbar)[9]) {",
         "  uint32_t q[9];",
         "  uint64_t cc;",
         _whole(lines, outs, ins, [f"v{ACC}", f"v{ACC + 1}"]),
         "}"]
    return "\n".join(o)


def gen_mont_whole():
    A = f"v[{ACC}:{ACC + 1}]"
    R, Mo, CC, Ai, Bi, P, PINV = 0, L, 2 * L, 2 * L + 1, 3 * L + 1, 4 * L + 1, 5 * L + 1
    lines = []
    for i in range(L):
        first = i == 0
        for j in range(i + 1):
            lines.append(f"v_mad_u64_u32 {A}, %{CC}, %{Ai + j}, %{Bi + i - j}, {'0' if first else A}")
            first = False
        for j in range(i):
            lines.append(f"v_mad_u64_u32 {A}, %{CC}, %{Mo + j}, %{P + i - j}, {A}")
        lines.append(f"v_mul_lo_u32 %{Mo + i}, v{ACC}, %{PINV}")
        lines.append(f"v_and_b32 %{Mo + i}, {MASK}, %{Mo + i}")
        lines.append(f"v_mad_u64_u32 {A}, %{CC}, %{Mo + i}, %{P}, {A}")
        lines.append(f"v_lshrrev_b64 {A}, 29, {A}")
    for i in range(L, 2 * L):
        for j in range(i - L + 1, L):
            lines.append(f"v_mad_u64_u32 {A}, %{CC}, %{Ai + j}, %{Bi + i - j}, {A}")
        for j in range(i - L + 1, L):
            lines.append(f"v_mad_u64_u32 {A}, %{CC}, %{Mo + j}, %{P + i - j}, {A}")
        lines.append(f"v_and_b32 %{R + i - L}, {MASK}, v{ACC}")
        if i + 1 < 2 * L:
            lines.append(f"v_lshrrev_b64 {A}, 29, {A}")
    outs = [f'"=&v"(r[{k}])' for k in range(L)] + [f'"=&v"(m[{k}])' for k in range(L)] + ['"=&s"(cc)']
    ins = ([f'"v"(a[{k}])' for k in range(L)] + [f'"v"(b[{k}])' for k in range(L)] +
           [f'"s"(M.p[{k}])' for k in range(L)] + ['"s"(M.pinv)'])
    o = ["__device__ __forceinline__ void mont29_a9(uint32_t (&r)[9], const uint32_t (&a)[9], const uint32_t (&b)[9],",
         "                                          const Mod29<9>& M) {",
         "  uint32_t m[9];",
         "  uint64_t cc;",
         _whole(lines, outs, ins, [f"v{ACC}", f"v{ACC + 1}"]),
         "}"]
    return "\n".join(o)


def main():
    # The checked-in header (ntt_amd/csrc/field29_asm9.hpp) holds the product form only.  The measured
    # alternatives stay here as generator options, for experiment builds:
    #   --whole  one asm statement per product (1.73 vs 1.67 ms at 2^24 BN254: spills, no ILP across products)
    #   --pair   two product columns per statement, their MAD chains interleaved (+2.0 %)
    variant = "whole" if "--whole" in sys.argv else ("pair" if "--pair" in sys.argv else "")
    print("// GENERATED by tools/gen_field29_asm.py" + (f" --{variant}" if variant else "") + " -- do not edit.")
    print("// L = 9 radix-2^29 products (field29.hpp mulc29 / mont29) with one inline-asm MAD chain per")
    print("// product column; see the generator for why.  Device only.")
    print("#pragma once")
    print('#include "field29.hpp"')
    print()
    print("namespace ntt {")
    if variant == "whole":
        print("#if defined(__HIP_DEVICE_COMPILE__)")
        print("// one asm statement per product (see the generator)")
        print(gen_mulc_whole())
        print()
        print(gen_mont_whole())
        print("__device__ __forceinline__ void mulc29_a9u(uint32_t (&r)[9], const uint32_t (&x)[9], const uint32_t (&w)[9],")
        print("                                           const uint32_t (&ws)[9], const uint32_t (&pbar)[9]) {")
        print("  mulc29_a9(r, x, w, ws, pbar);")
        print("}")
    elif variant == "pair":
        print("#if defined(__HIP_DEVICE_COMPILE__)")
        print("// two product columns per asm statement, their MAD chains interleaved (see the generator)")
        print(gen_mulc_pair())
        print()
        print(gen_mulc_pair(uniform=True))
        print()
        print(gen_mont())
    else:
        print("#if defined(__HIP_DEVICE_COMPILE__)")
        print("// one asm statement per product column")
        print(gen_mulc())
        print()
        print(gen_mulc(uniform=True))
        print()
        print(gen_mont())
    print("#else  // host pass: the generic forms (same results)")
    print("F29_HD void mulc29_a9(uint32_t (&r)[9], const uint32_t (&x)[9], const uint32_t (&w)[9], const uint32_t (&ws)[9],")
    print("                       const uint32_t (&pbar)[9]) {")
    print("  mulc29<9>(r, x, w, ws, pbar);")
    print("}")
    print("F29_HD void mulc29_a9u(uint32_t (&r)[9], const uint32_t (&x)[9], const uint32_t (&w)[9], const uint32_t (&ws)[9],")
    print("                        const uint32_t (&pbar)[9]) {")
    print("  mulc29<9>(r, x, w, ws, pbar);")
    print("}")
    print("F29_HD void mont29_a9(uint32_t (&r)[9], const uint32_t (&a)[9], const uint32_t (&b)[9], const Mod29<9>& M) {")
    print("  mont29<9>(r, a, b, M);")
    print("}")
    print("#endif")
    print("}  // namespace ntt")


if __name__ == "__main__":
    main()
