"""Generate korali_amd/csrc/kg_chains.hpp: the ordered FP64 chains of the
GSL-order tridiagonalisation as hand-scheduled gfx950 inline assembly.

Why assembly: an ordered double-precision sum is a chain of dependent
v_add_f64.  Measured on MI355X (tools/ubench_chains.hip): ONE wave issues a
v_add_f64 every ~9.3 cycles whether or not the adds depend on each other
(4 independent chains: 9.8 cycles per add), so a chain is bound by the
instruction count of the wave that runs it, ~8-10 cycles per instruction of
any kind.  These loops therefore carry nothing but the adds, one ds_read2
per two elements and a few scalar instructions per 16 (kc_add: 15.4 cycles
per element alone; the compiler's schedule of the same C++ waited and
branched per element: 20-44).

Each primitive runs whole groups (8 or 16 elements) and relies on the caller
padding the staged values with +0.0 (an exact no-op for every chain here:
the accumulators never hold -0.0), so there is no tail code.  Loads run up
to one group past the last element; callers keep that slack inside LDS.

Scratch registers v[192:255] are declared clobbered; kernels using these
primitives are compiled for at most 512 threads per workgroup (256 VGPRs).

Run: python tools/gen_chains.py  (rewrites the header; commit both).
"""
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "korali_amd", "csrc", "kg_chains.hpp")
OUT_EXP = os.path.join(ROOT, "tools", "kg_chains_experimental.hpp")

S0 = 192  # first scratch VGPR


def d(i):
    """double in scratch slot i (two VGPRs)"""
    return f"v[{S0 + 2 * i}:{S0 + 2 * i + 1}]"


def q(i):
    """slots 2i, 2i+1 as one ds_read2_b64 destination"""
    return f"v[{S0 + 4 * i}:{S0 + 4 * i + 3}]"


CLOBBER = ", ".join(f'"v{r}"' for r in range(S0, 256))


def asm_block(lines):
    return "\n".join(f'      "{ln}\\n"' for ln in lines)


def emit_add():
    """acc + p[0] + ... + p[16 g - 1]; slots 0-7 = set A, 8-15 = set B"""
    L = ["s_cmp_eq_u32 %[g], 0", "s_cbranch_scc1 9f"]
    for k in range(8):  # prologue: A = elements 0..7, B = 8..15
        L.append(f"ds_read2_b64 {q(k)}, %[p] offset0:{2 * k} offset1:{2 * k + 1}")
    L.append("1:")
    for half in range(2):  # A then B
        L.append("s_waitcnt lgkmcnt(4)")
        for t in range(8):
            L.append(f"v_add_f64 %[acc], %[acc], {d(8 * half + t)}")
            if t % 2 == 1:  # the pair just consumed: reload it 16 elements ahead
                k = 4 * half + t // 2
                L.append(f"ds_read2_b64 {q(k)}, %[p] offset0:{16 + 2 * k} offset1:{17 + 2 * k}")
            if half == 0 and t == 3:
                L.append("s_sub_u32 %[g], %[g], 1")
        if half == 1:
            pass
    L += ["v_add_u32 %[p], 0x80, %[p]", "s_cmp_lg_u32 %[g], 0", "s_cbranch_scc1 1b", "9:", "s_waitcnt lgkmcnt(0)"]
    return f"""
// acc + p[0] + ... + p[16 g - 1] in order (p: LDS byte address, wave-uniform)
__device__ __forceinline__ double kc_add(double acc, unsigned p, unsigned g) {{
  asm volatile(
{asm_block(L)}
      : [acc] "+&v"(acc), [p] "+&v"(p), [g] "+&s"(g)
      :
      : "scc", "memory", {CLOBBER});
  return acc;
}}
"""


def emit_add_desc():
    """acc + p[top] + p[top-1] + ... over 16 g elements; one 16-element
    group of loads in flight (set A: slots 0-15, set B: slots 16-31)."""
    def load(setb):
        s = 8 if setb else 0
        out = [f"ds_read2_b64 {q(s + k)}, %[p] offset0:{15 - 2 * k} offset1:{14 - 2 * k}" for k in range(8)]
        out.append("v_add_u32 %[p], 0xffffff80, %[p]")
        return out

    def proc(setb, loads):
        s = 16 if setb else 0
        out = ["s_waitcnt lgkmcnt(0)"]
        for t in range(16):
            out.append(f"v_add_f64 %[acc], %[acc], {d(s + t)}")
            if t < len(loads):
                out.append(loads[t])
        return out

    L = ["s_cmp_eq_u32 %[g], 0", "s_cbranch_scc1 9f"] + load(False)
    L.append("1:")
    L += proc(False, load(True))
    L += ["s_sub_u32 %[g], %[g], 1", "s_cmp_eq_u32 %[g], 0", "s_cbranch_scc1 9f"]
    L += proc(True, load(False))
    L += ["s_sub_u32 %[g], %[g], 1", "s_cmp_lg_u32 %[g], 0", "s_cbranch_scc1 1b", "9:", "s_waitcnt lgkmcnt(0)"]
    return f"""
// acc + p[top] + p[top-1] + ... over 16 g elements in that order (gslcblas
// dsymv's descending walk over staged products); p = LDS byte address of
// element top-15 (wave-uniform); the loads run one group below the last
// element
__device__ __forceinline__ double kc_add_desc(double acc, unsigned p, unsigned g) {{
  asm volatile(
{asm_block(L)}
      : [acc] "+&v"(acc), [p] "+&v"(p), [g] "+&s"(g)
      :
      : "scc", "memory", {CLOBBER});
  return acc;
}}
"""


def emit_nrm2():
    """gslcblas dnrm2's ssq recurrence over a block of up to 128 elements,
    fully unrolled (static LDS offsets, no address updates): element e is
    ssq += t_e, or (mask bit e set: a new running maximum) ssq = 1 + ssq t_e
    t_e.  Per 8-element half-group: one s_and_b32 on its 32-bit mask word
    (SCC = any rescale) and a branch; a half without rescales is 8 plain adds,
    a half with them tests each element (rescale bodies out of line).  The
    block ends after 16 g elements (one s_cmp + branch per 16)."""
    L = []
    words = ["%[k0l]", "%[k0h]", "%[k1l]", "%[k1h]"]
    for k in range(8):  # halves 0, 1 in flight
        L.append(f"ds_read2_b64 {q(k)}, %[p] offset0:{2 * k} offset1:{2 * k + 1}")
    slow = []
    for hf in range(16):
        st = 8 * (hf % 2)  # register slots of this half
        w, sh = words[hf // 4], 8 * (hf % 4)
        if hf % 2 == 0:
            L += ["s_cmp_eq_u32 %[g], 0", "s_cbranch_scc1 9f", "s_sub_u32 %[g], %[g], 1"]
        L.append("s_waitcnt lgkmcnt(4)")
        L += [f"s_and_b32 %[t], {w}, {hex(0xff << sh)}", f"s_cbranch_scc1 {100 + hf}f"]
        nxt = [f"ds_read2_b64 {q(4 * (hf % 2) + k)}, %[p] offset0:{16 * (hf // 2 + 1) + 8 * (hf % 2) + 2 * k} "
               f"offset1:{16 * (hf // 2 + 1) + 8 * (hf % 2) + 2 * k + 1}" for k in range(4)]
        for t in range(8):
            L.append(f"v_add_f64 %[acc], %[acc], {d(st + t)}")
            if t % 2 == 1:
                L.append(nxt[t // 2])
        L.append(f"{200 + hf}:")
        # out-of-line slow half
        slow.append(f"{100 + hf}:")
        for t in range(8):
            slow += [f"s_bitcmp1_b32 {w}, {sh + t}", f"s_cbranch_scc1 {300 + 8 * hf + t}f",
                     f"v_add_f64 %[acc], %[acc], {d(st + t)}", f"{500 + 8 * hf + t}:"]
        slow += nxt + [f"s_branch {200 + hf}b"]
        for t in range(8):
            slow += [f"{300 + 8 * hf + t}:",
                     f"v_mul_f64 %[tmp], %[acc], {d(st + t)}", f"v_mul_f64 %[tmp], %[tmp], {d(st + t)}",
                     "v_add_f64 %[acc], 1.0, %[tmp]", f"s_branch {500 + 8 * hf + t}b"]
    L += ["s_branch 9f"] + slow + ["9:", "s_waitcnt lgkmcnt(0)"]
    return f"""
// gslcblas dnrm2's ssq recurrence over p[0 .. 16 g) (g <= 8): element e is a
// new running maximum where bit e of the 128-bit mask (k1h:k1l:k0h:k0l) is
// set, ssq = 1 + (ssq t) t, else ssq += t (GSL's operation order; SURVEY.md
// Appendix A).  Loads run 16 elements past the block.
__device__ __forceinline__ double kc_nrm2(double acc, unsigned p, unsigned g, unsigned long long k0,
                                          unsigned long long k1) {{
  const unsigned k0l = __builtin_amdgcn_readfirstlane((unsigned)k0), k0h = __builtin_amdgcn_readfirstlane((unsigned)(k0 >> 32));
  const unsigned k1l = __builtin_amdgcn_readfirstlane((unsigned)k1), k1h = __builtin_amdgcn_readfirstlane((unsigned)(k1 >> 32));
  unsigned t;
  double tmp;
  asm volatile(
{asm_block(L)}
      : [acc] "+&v"(acc), [g] "+&s"(g), [t] "=&s"(t), [tmp] "=&v"(tmp)
      : [p] "v"(p), [k0l] "s"(k0l), [k0h] "s"(k0h), [k1l] "s"(k1l), [k1h] "s"(k1h)
      : "scc", "memory", {CLOBBER});
  return acc;
}}
"""


def emit_lock(desc):
    """Lockstep per-lane chains acc_lane + sum_t w_t m_t (each product
    rounded, then added): w wave-uniform (broadcast LDS reads), m per lane.
    8-element batches, the next batch's loads in flight while the current
    one is multiplied and added (set A: w slots 0-7, m 8-15; set B: w
    16-23, m 24-31).  Pairs of elements come in one ds_read_b128 (4 LDS
    cycles per wave-instruction, 256 B/clk; ds_read2_b64 takes 8 for the same
    16 bytes per lane, MI355X_MICROARCH.md §LDS): w always, m of the
    descending walk (two consecutive columns of the row); the ascending
    walk's m is a column (one ds_read_b64 per element, 2 cycles).  Callers
    keep every pair 16-byte aligned."""

    def load(setb):
        ws, ms = (16, 24) if setb else (0, 8)
        out = []
        for k in range(4):
            if desc:  # element t at byte offset (7 - t) * 8 above the batch base: pair k = offsets 6-2k, 7-2k
                out.append(f"ds_read_b128 {q(ws // 2 + k)}, %[pw] offset:{(6 - 2 * k) * 8}")
                out.append(f"ds_read_b128 {q(ms // 2 + k)}, %[pm] offset:{(6 - 2 * k) * 8}")
            else:
                out.append(f"ds_read_b128 {q(ws // 2 + k)}, %[pw] offset:{16 * k}")
                out.append(f"ds_read_b64 {d(ms + 2 * k)}, %[pm] offset:%[o{2 * k}]")
                out.append(f"ds_read_b64 {d(ms + 2 * k + 1)}, %[pm] offset:%[o{2 * k + 1}]")
        if desc:
            out.append("v_add_u32 %[pw], 0xffffffc0, %[pw]")
            out.append("v_add_u32 %[pm], 0xffffffc0, %[pm]")
        else:
            out.append("v_add_u32 %[pw], 0x40, %[pw]")
            out.append("v_add_u32 %[pm], %[s8], %[pm]")
        return out

    def proc(setb, loads):
        ws, ms = (16, 24) if setb else (0, 8)
        out = ["s_waitcnt lgkmcnt(0)"]
        li = 0
        per = (len(loads) + 7) // 8
        for t in range(8):
            sl = (t ^ 1) if desc else t  # descending: the pair's high element (the higher column) first
            out.append(f"v_mul_f64 {d(ws + sl)}, {d(ws + sl)}, {d(ms + sl)}")
            for _ in range(per):  # the other set's loads fill this batch's stall slots
                if li < len(loads):
                    out.append(loads[li])
                    li += 1
            out.append(f"v_add_f64 %[acc], %[acc], {d(ws + sl)}")
        out += loads[li:]
        return out

    L = ["s_cmp_eq_u32 %[nb], 0", "s_cbranch_scc1 9f"]
    L += load(False)
    L.append("1:")
    L += proc(False, load(True))
    L += ["s_sub_u32 %[nb], %[nb], 1", "s_cmp_eq_u32 %[nb], 0", "s_cbranch_scc1 9f"]
    L += proc(True, load(False))
    L += ["s_sub_u32 %[nb], %[nb], 1", "s_cmp_lg_u32 %[nb], 0", "s_cbranch_scc1 1b", "9:", "s_waitcnt lgkmcnt(0)"]
    body = asm_block(L)
    if desc:
        return f"""
// per-lane chain acc + w[top] m[top] + w[top-1] m[top-1] + ... over 8 nb
// elements (each product rounded, then added: gslcblas dsymv's descending
// column walk).  pw / pm = LDS byte addresses of element top-7 (w uniform,
// m per lane), both 16-byte aligned; the loads run one batch below the last
// element.
__device__ __forceinline__ double kc_lock_desc(double acc, unsigned pw, unsigned pm, unsigned nb) {{
  asm volatile(
{body}
      : [acc] "+&v"(acc), [pw] "+&v"(pw), [pm] "+&v"(pm), [nb] "+&s"(nb)
      :
      : "scc", "memory", {CLOBBER});
  return acc;
}}
"""
    offs = ", ".join(f'[o{t}] "i"({t} * S)' for t in range(8))
    return f"""
// per-lane chain acc + w[0] m[0] + w[1] m[S] + w[2] m[2 S] + ... over 8 nb
// elements (gslcblas dsymv's ascending t2 walk).  pw = LDS byte address of
// w[0] (uniform, 16-byte aligned), pm = per-lane LDS byte address of m[0],
// S = the m stride in bytes; the loads run one batch past the last element.
template <int S>
__device__ __forceinline__ double kc_lock_asc(double acc, unsigned pw, unsigned pm, unsigned nb) {{
  asm volatile(
{body}
      : [acc] "+&v"(acc), [pw] "+&v"(pw), [pm] "+&v"(pm), [nb] "+&s"(nb)
      : [s8] "i"(8 * S), {offs}
      : "scc", "memory", {CLOBBER});
  return acc;
}}
"""


def emit_lock_dpp(desc):
    """Lockstep per-lane chains as emit_lock, but w reaches every lane through
    a DPP broadcast from a register instead of a broadcast LDS read: per
    8-element batch one ds_read_b64 brings w[base + (lane & 7)] into W (each
    16-lane row holds the batch's 8 values in lanes 0-7), v_mov_b64 ...
    row_newbcast:j copies element j to every lane, then the rounded product
    and the ordered add.  LDS traffic per element and wave: m only (a b128 pair
    per two elements descending, a b64 per element ascending) + 1/8 of a b64.
    Set A: W v[192:193], m slots v[194:209]; set B: W v[210:211], m v[212:227];
    broadcast temporaries v[228:231]."""
    WA, MA, WB, MB, XT = 192, 194, 210, 212, 228

    def ms(mb, sl):
        return f"v[{mb + 2 * sl}:{mb + 2 * sl + 1}]"

    def load(setb):
        w, m = (WB, MB) if setb else (WA, MA)
        out = [f"ds_read_b64 v[{w}:{w + 1}], %[pwl]"]
        for k in range(4):
            if desc:  # pair p = 3 - k: columns base + 2p (slot 2p) and base + 2p + 1 (slot 2p + 1), top pair first
                pp = 3 - k
                out.append(f"ds_read_b128 v[{m + 4 * pp}:{m + 4 * pp + 3}], %[pm] offset:{16 * pp}")
            else:
                out.append(f"ds_read_b64 {ms(m, 2 * k)}, %[pm] offset:%[o{2 * k}]")
                out.append(f"ds_read_b64 {ms(m, 2 * k + 1)}, %[pm] offset:%[o{2 * k + 1}]")
        if desc:
            out += ["v_add_u32 %[pwl], 0xffffffc0, %[pwl]", "v_add_u32 %[pm], 0xffffffc0, %[pm]"]
        else:
            out += ["v_add_u32 %[pwl], 0x40, %[pwl]", "v_add_u32 %[pm], %[s8], %[pm]"]
        return out

    def proc(setb, loads):
        w, m = (WB, MB) if setb else (WA, MA)
        out = ["s_waitcnt lgkmcnt(0)"]
        li = 0
        per = (len(loads) + 7) // 8
        for t in range(8):
            # descending: element t is column base + 7 - t (lane 7 - t of W; m slot (7 - t) in the pairs)
            j = 7 - t if desc else t
            sl = j  # slot s holds column base + s (both walks)
            x = f"v[{XT + 2 * (t % 2)}:{XT + 2 * (t % 2) + 1}]"
            out.append(f"v_mov_b64 {x}, v[{w}:{w + 1}] row_newbcast:{j} row_mask:0xf bank_mask:0xf")
            for _ in range(per):
                if li < len(loads):
                    out.append(loads[li])
                    li += 1
            out.append(f"v_mul_f64 {ms(m, sl)}, {x}, {ms(m, sl)}")
            out.append(f"v_add_f64 %[acc], %[acc], {ms(m, sl)}")
        out += loads[li:]
        return out

    L = ["s_cmp_eq_u32 %[nb], 0", "s_cbranch_scc1 9f"]
    L += load(False)
    L.append("1:")
    L += proc(False, load(True))
    L += ["s_sub_u32 %[nb], %[nb], 1", "s_cmp_eq_u32 %[nb], 0", "s_cbranch_scc1 9f"]
    L += proc(True, load(False))
    L += ["s_sub_u32 %[nb], %[nb], 1", "s_cmp_lg_u32 %[nb], 0", "s_cbranch_scc1 1b", "9:", "s_waitcnt lgkmcnt(0)"]
    body = asm_block(L)
    clob = ", ".join(f'"v{r}"' for r in range(192, 232))
    if desc:
        return f"""
// kc_lock_desc with w broadcast from registers (DPP): pwl = per-lane LDS byte
// address of w[top - 7 + (lane & 7)], pm = per-lane address of m[top - 7]
// (16-byte aligned)
__device__ __forceinline__ double kc_lock_desc_dpp(double acc, unsigned pwl, unsigned pm, unsigned nb) {{
  asm volatile(
{body}
      : [acc] "+&v"(acc), [pwl] "+&v"(pwl), [pm] "+&v"(pm), [nb] "+&s"(nb)
      :
      : "scc", "memory", {clob});
  return acc;
}}
"""
    offs = ", ".join(f'[o{t}] "i"({t} * S)' for t in range(8))
    return f"""
// kc_lock_asc with w broadcast from registers (DPP): pwl = per-lane LDS byte
// address of w[lane & 7], pm = per-lane address of m[0], S the m stride
template <int S>
__device__ __forceinline__ double kc_lock_asc_dpp(double acc, unsigned pwl, unsigned pm, unsigned nb) {{
  asm volatile(
{body}
      : [acc] "+&v"(acc), [pwl] "+&v"(pwl), [pm] "+&v"(pm), [nb] "+&s"(nb)
      : [s8] "i"(8 * S), {offs}
      : "scc", "memory", {clob});
  return acc;
}}
"""


def emit_dpp_chains():
    """Chains over staged values held in REGISTERS: element 16 k + j sits in
    lane j of every row of q[k] (8 VGPR pairs, 128 elements) and reaches the
    accumulator through a DPP row_newbcast:j operand of v_fmac_f64 (acc = q *
    1.0 + acc: the product is exact, so this is acc + q rounded once, the
    same IEEE add as v_add_f64).  No memory operation inside the chain: one
    VALU instruction per element (kc_add's ds_read2 per two elements, its
    lgkmcnt waits and the LDS traffic of other waves are gone)."""
    qs = ", ".join(f"[q{k}] \"v\"(q[{k}])" for k in range(8))

    def fast(e):
        k, j = e // 16, e % 16
        return f"v_fmac_f64 %[acc], %[q{k}], %[one] row_newbcast:{j} row_mask:0xf bank_mask:0xf"

    # plain ordered sum (s_nop 1: the two wait states between a VALU write of
    # a DPP source and its DPP read, in case the compiler formed q by VALU)
    L = ["s_nop 1"]
    for grp in range(8):
        L += ["s_cmp_eq_u32 %[g], 0", "s_cbranch_scc1 9f", "s_sub_u32 %[g], %[g], 1"]
        L += [fast(16 * grp + t) for t in range(16)]
    L += ["9:"]
    add = f"""
// acc + e_0 + e_1 + ... + e_(16 g - 1) in order, e_(16 k + j) = lane j of q[k]
// (g <= 8; elements past the block are +0.0 no-ops)
__device__ __forceinline__ double kc_add_dpp(double acc, const double (&q)[8], unsigned g) {{
  const double one = 1.0;
  asm volatile(
{asm_block(L)}
      : [acc] "+&v"(acc), [g] "+&s"(g)
      : {qs}, [one] "v"(one)
      : "scc");
  return acc;
}}
"""
    # dnrm2's ssq recurrence with the rescale mask (as kc_nrm2)
    words = ["%[k0l]", "%[k0h]", "%[k1l]", "%[k1h]"]
    L = ["s_nop 1"]
    slow = []
    for hf in range(16):
        w, sh = words[hf // 4], 8 * (hf % 4)
        if hf % 2 == 0:
            L += ["s_cmp_eq_u32 %[g], 0", "s_cbranch_scc1 9f", "s_sub_u32 %[g], %[g], 1"]
        L += [f"s_and_b32 %[t], {w}, {hex(0xff << sh)}", f"s_cbranch_scc1 {100 + hf}f"]
        L += [fast(8 * hf + t) for t in range(8)]
        L.append(f"{200 + hf}:")
        slow.append(f"{100 + hf}:")
        for t in range(8):
            e = 8 * hf + t
            k, j = e // 16, e % 16
            slow += [f"s_bitcmp1_b32 {w}, {sh + t}", f"s_cbranch_scc1 {300 + e}f", fast(e), f"{500 + e}:"]
        slow += [f"s_branch {200 + hf}b"]
        for t in range(8):
            e = 8 * hf + t
            k, j = e // 16, e % 16
            slow += [f"{300 + e}:",
                     f"v_mov_b64 %[x], %[q{k}] row_newbcast:{j} row_mask:0xf bank_mask:0xf",
                     "v_mul_f64 %[tmp], %[acc], %[x]", "v_mul_f64 %[tmp], %[tmp], %[x]",
                     "v_add_f64 %[acc], 1.0, %[tmp]", f"s_branch {500 + e}b"]
    L += ["s_branch 9f"] + slow + ["9:"]
    nrm2 = f"""
// gslcblas dnrm2's ssq recurrence over e_0 .. e_(16 g - 1) (g <= 8), the
// elements in registers as kc_add_dpp: where bit e of the 128-bit mask is
// set, ssq = 1 + (ssq t) t, else ssq += t (as kc_nrm2)
__device__ __forceinline__ double kc_nrm2_dpp(double acc, const double (&q)[8], unsigned g, unsigned long long k0,
                                              unsigned long long k1) {{
  const unsigned k0l = __builtin_amdgcn_readfirstlane((unsigned)k0), k0h = __builtin_amdgcn_readfirstlane((unsigned)(k0 >> 32));
  const unsigned k1l = __builtin_amdgcn_readfirstlane((unsigned)k1), k1h = __builtin_amdgcn_readfirstlane((unsigned)(k1 >> 32));
  const double one = 1.0;
  unsigned t;
  double tmp, x;
  asm volatile(
{asm_block(L)}
      : [acc] "+&v"(acc), [g] "+&s"(g), [t] "=&s"(t), [tmp] "=&v"(tmp), [x] "=&v"(x)
      : {qs}, [one] "v"(one), [k0l] "s"(k0l), [k0h] "s"(k0h), [k1l] "s"(k1l), [k1h] "s"(k1h)
      : "scc");
  return acc;
}}
"""
    # one row chain step-group: every 16-lane row adds its own lanes 0..15 of q
    L = ["s_nop 1"] + [f"v_fmac_f64 %[acc], %[q], %[one] row_newbcast:{j} row_mask:0xf bank_mask:0xf"
                       for j in range(16)]
    row16 = f"""
// ROW chains: each 16-lane row r of the wave keeps its own accumulator and
// adds lanes 16 r + 0, ..., 16 r + 15 of q in that order (four independent
// ordered chains per wave, one VALU instruction per element)
__device__ __forceinline__ double kc_row16(double acc, double q) {{
  const double one = 1.0;
  asm volatile(
{asm_block(L)}
      : [acc] "+&v"(acc)
      : [q] "v"(q), [one] "v"(one));
  return acc;
}}
"""
    # experimental forms of the ssq recurrence (tools/ubench_chains.hip modes
    # 21-25 compare them with kc_nrm2_dpp):
    # (1) per-element check: every element tests its mask bit (no half-level
    #     fast path), the rescale bodies out of line
    L = ["s_nop 1"]
    slow = []
    for e in range(128):
        k, j = e // 16, e % 16
        w, b = words[e // 32], e % 32
        if e % 16 == 0:
            L += ["s_cmp_eq_u32 %[g], 0", "s_cbranch_scc1 9f", "s_sub_u32 %[g], %[g], 1"]
        L += [f"s_bitcmp1_b32 {w}, {b}", f"s_cbranch_scc1 {300 + e}f", fast(e), f"{500 + e}:"]
        slow += [f"{300 + e}:", f"v_mov_b64 %[x], %[q{k}] row_newbcast:{j} row_mask:0xf bank_mask:0xf",
                 "v_mul_f64 %[tmp], %[acc], %[x]", "v_mul_f64 %[tmp], %[tmp], %[x]",
                 "v_add_f64 %[acc], 1.0, %[tmp]", f"s_branch {500 + e}b"]
    L += ["s_branch 9f"] + slow + ["9:"]
    nrm2c = f"""
// (experimental) kc_nrm2_dpp with a mask test per element instead of per half
__device__ __forceinline__ double kc_nrm2_dppc(double acc, const double (&q)[8], unsigned g, unsigned long long k0,
                                               unsigned long long k1) {{
  const unsigned k0l = __builtin_amdgcn_readfirstlane((unsigned)k0), k0h = __builtin_amdgcn_readfirstlane((unsigned)(k0 >> 32));
  const unsigned k1l = __builtin_amdgcn_readfirstlane((unsigned)k1), k1h = __builtin_amdgcn_readfirstlane((unsigned)(k1 >> 32));
  const double one = 1.0;
  double tmp, x;
  asm volatile(
{asm_block(L)}
      : [acc] "+&v"(acc), [g] "+&s"(g), [tmp] "=&v"(tmp), [x] "=&v"(x)
      : {qs}, [one] "v"(one), [k0l] "s"(k0l), [k0h] "s"(k0h), [k1l] "s"(k1l), [k1h] "s"(k1h)
      : "scc");
  return acc;
}}
"""
    # (2) branch-free: every element as u = ssq a, w = u a, ssq = w + c with
    #     (a, c) = (t, 1) at a new running maximum and (1, t) elsewhere (ssq
    #     times 1.0 is exact, so a plain element is ssq + t rounded once)
    qa = ", ".join(f"[a{k}] \"v\"(a[{k}])" for k in range(8))
    qc = ", ".join(f"[c{k}] \"v\"(c[{k}])" for k in range(8))
    L = ["s_nop 1"]
    for e in range(128):
        k, j = e // 16, e % 16
        if e % 16 == 0:
            L += ["s_cmp_eq_u32 %[g], 0", "s_cbranch_scc1 9f", "s_sub_u32 %[g], %[g], 1"]
        L += [f"v_mov_b64 %[xa], %[a{k}] row_newbcast:{j} row_mask:0xf bank_mask:0xf",
              f"v_mov_b64 %[xc], %[c{k}] row_newbcast:{j} row_mask:0xf bank_mask:0xf",
              "v_mul_f64 %[tmp], %[acc], %[xa]", "v_mul_f64 %[tmp], %[tmp], %[xa]", "v_add_f64 %[acc], %[tmp], %[xc]"]
    L += ["9:"]
    nrm23 = f"""
// (experimental) the branch-free three-operation form of the ssq recurrence
__device__ __forceinline__ double kc_nrm2_dpp3(double acc, const double (&a)[8], const double (&c)[8], unsigned g) {{
  double tmp, xa, xc;
  asm volatile(
{asm_block(L)}
      : [acc] "+&v"(acc), [g] "+&s"(g), [tmp] "=&v"(tmp), [xa] "=&v"(xa), [xc] "=&v"(xc)
      : {qa}, {qc}
      : "scc");
  return acc;
}}
"""
    # (3) kc_nrm2_dpp with the branch-free three-operation form for the
    #     halves (H = 8) or quarters (H = 4) that hold a rescale: a span
    #     without one is H plain DPP adds of c, a span with one runs
    #     u = ssq a, w = u a, ssq = w + c on every element, straight-line
    def spans(H, name):
        L = ["s_nop 1"]
        slow = []
        nsp = 128 // H
        for hf in range(nsp):
            w, sh = words[(hf * H) // 32], (hf * H) % 32
            if (hf * H) % 16 == 0:
                L += ["s_cmp_eq_u32 %[g], 0", "s_cbranch_scc1 9f", "s_sub_u32 %[g], %[g], 1"]
            L += [f"s_and_b32 %[t], {w}, {hex(((1 << H) - 1) << sh)}", f"s_cbranch_scc1 {100 + hf}f"]
            for t in range(H):
                e = H * hf + t
                k, j = e // 16, e % 16
                L.append(f"v_fmac_f64 %[acc], %[c{k}], %[one] row_newbcast:{j} row_mask:0xf bank_mask:0xf")
            L.append(f"{200 + hf}:")
            slow.append(f"{100 + hf}:")
            for t in range(H):
                e = H * hf + t
                k, j = e // 16, e % 16
                slow += [f"v_mov_b64 %[xa], %[a{k}] row_newbcast:{j} row_mask:0xf bank_mask:0xf",
                         f"v_mov_b64 %[xc], %[c{k}] row_newbcast:{j} row_mask:0xf bank_mask:0xf",
                         "v_mul_f64 %[tmp], %[acc], %[xa]", "v_mul_f64 %[tmp], %[tmp], %[xa]",
                         "v_add_f64 %[acc], %[tmp], %[xc]"]
            slow += [f"s_branch {200 + hf}b"]
        L += ["s_branch 9f"] + slow + ["9:"]
        return f"""
// (experimental) kc_nrm2_dpp over {H}-element spans, a span holding a rescale
// in the branch-free three-operation form; a[] = t at a new running maximum,
// else 1.0; c[] = 1.0 there, else t
__device__ __forceinline__ double {name}(double acc, const double (&a)[8], const double (&c)[8], unsigned g,
                                         unsigned long long k0, unsigned long long k1) {{
  const unsigned k0l = __builtin_amdgcn_readfirstlane((unsigned)k0), k0h = __builtin_amdgcn_readfirstlane((unsigned)(k0 >> 32));
  const unsigned k1l = __builtin_amdgcn_readfirstlane((unsigned)k1), k1h = __builtin_amdgcn_readfirstlane((unsigned)(k1 >> 32));
  const double one = 1.0;
  unsigned t;
  double tmp, xa, xc;
  asm volatile(
{asm_block(L)}
      : [acc] "+&v"(acc), [g] "+&s"(g), [t] "=&s"(t), [tmp] "=&v"(tmp), [xa] "=&v"(xa), [xc] "=&v"(xc)
      : {qa}, {qc}, [one] "v"(one), [k0l] "s"(k0l), [k0h] "s"(k0h), [k1l] "s"(k1l), [k1h] "s"(k1h)
      : "scc");
  return acc;
}}
"""
    # the product calls kc_add_dpp, kc_row16 and kc_nrm2_dpp8; the other forms
    # are measured by tools/ubench_chains.hip / checked by check_dpp_chains.hip
    return (add + row16 + spans(8, "kc_nrm2_dpp8"),
            nrm2 + nrm2c + nrm23 + spans(4, "kc_nrm2_dpp4"))


def main():
    dpp_product, dpp_experimental = emit_dpp_chains()
    hdr = f"""// kg_chains.hpp — GENERATED by tools/gen_chains.py; do not edit.
//
// Ordered FP64 chains of the GSL-order tridiagonalisation as hand-scheduled
// gfx950 assembly (see the generator's docstring for why and how).  Every
// chain keeps the reference's operation order; +,* are IEEE correctly
// rounded on gfx950, so the results equal the oracle's bit for bit.  Only the
// forms the product kernels call live here; the measured alternatives are in
// tools/kg_chains_experimental.hpp.
#pragma once
namespace kg {{
namespace chains {{
{emit_add()}{emit_add_desc()}{emit_nrm2()}{emit_lock(True)}{emit_lock(False)}{dpp_product}
}}  // namespace chains
}}  // namespace kg
"""
    with open(OUT, "w") as f:
        f.write(hdr)
    print("wrote", OUT)
    exp = f"""// kg_chains_experimental.hpp — GENERATED by tools/gen_chains.py; do not edit.
//
// Chain forms measured against the product's (tools/ubench_chains.hip,
// tools/check_dpp_chains.hip) and not called by any product kernel:
// the DPP lockstep forms, the per-half / per-
// element / branch-free / quarter-span variants of the dnrm2 recurrence.
// Include after korali_amd/csrc/kg_chains.hpp.
#pragma once
namespace kg {{
namespace chains {{
{emit_lock_dpp(True)}{emit_lock_dpp(False)}{dpp_experimental}
}}  // namespace chains
}}  // namespace kg
"""
    with open(OUT_EXP, "w") as f:
        f.write(exp)
    print("wrote", OUT_EXP)


if __name__ == "__main__":
    main()
