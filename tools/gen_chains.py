"""Generate korali_amd/csrc/kg_chains.hpp: the ordered FP64 chains of the
GSL-order tridiagonalisation as hand-scheduled gfx950 inline assembly.

Why assembly: an ordered double-precision sum is a chain of dependent
v_add_f64 (8.3 cycles each on MI355X).  A wave issues at most one
instruction per 4-cycle slot, so everything else the chain needs (its LDS
loads, address updates, loop control) has to sit in the stall slots between
two dependent adds, and no wait may stand in front of an add whose operand
landed long ago.  The compiler's schedule for the same C++ waited before
every add and branched per element (kg_eigen.hip's round-2 kernels: 20-44
cycles per element); these loops issue 1.5-3.5 instructions per element.

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
      : [acc] "+v"(acc), [p] "+v"(p), [g] "+s"(g)
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
      : [acc] "+v"(acc), [p] "+v"(p), [g] "+s"(g)
      :
      : "scc", "memory", {CLOBBER});
  return acc;
}}
"""


def emit_nrm2():
    """gslcblas dnrm2's ssq recurrence: element e is ssq += t_e, or (mask bit
    e set: a new running maximum) ssq = 1 + ssq t_e t_e.  Groups of 16; the
    16 mask bits of a group select the fast (adds only) or the slow path."""
    L = ["s_cmp_eq_u32 %[g], 0", "s_cbranch_scc1 9f",
         "s_mov_b64 %[m], %[k0]", "s_mov_b32 %[wc], 4"]
    for k in range(8):
        L.append(f"ds_read2_b64 {q(k)}, %[p] offset0:{2 * k} offset1:{2 * k + 1}")
    L.append("1:")
    L += ["s_and_b64 %[t], %[m], 0xffff", "s_lshr_b64 %[m], %[m], 16", "s_cmp_eq_u64 %[t], 0", "s_cbranch_scc0 5f"]
    # fast path: 16 plain adds, reloads interleaved (as kc_add)
    for half in range(2):
        L.append("s_waitcnt lgkmcnt(4)")
        for t in range(8):
            L.append(f"v_add_f64 %[acc], %[acc], {d(8 * half + t)}")
            if t % 2 == 1:
                k = 4 * half + t // 2
                L.append(f"ds_read2_b64 {q(k)}, %[p] offset0:{16 + 2 * k} offset1:{17 + 2 * k}")
    L.append("s_branch 6f")
    # slow path: per-element test of the mask bit, reloads after the group
    L.append("5:")
    L.append("s_waitcnt lgkmcnt(4)")
    for u in range(16):
        if u == 8:
            L.append("s_waitcnt lgkmcnt(0)")
        L += [f"s_bitcmp1_b64 %[t], {u}", f"s_cbranch_scc1 {20 + u}f",
              f"v_add_f64 %[acc], %[acc], {d(u)}", f"s_branch {40 + u}f",
              f"{20 + u}:",
              f"v_mul_f64 %[tmp], %[acc], {d(u)}", f"v_mul_f64 %[tmp], %[tmp], {d(u)}",
              "v_add_f64 %[acc], 1.0, %[tmp]",
              f"{40 + u}:"]
    for k in range(8):
        L.append(f"ds_read2_b64 {q(k)}, %[p] offset0:{16 + 2 * k} offset1:{17 + 2 * k}")
    L.append("6:")
    L += ["v_add_u32 %[p], 0x80, %[p]",
          "s_sub_u32 %[g], %[g], 1", "s_cmp_eq_u32 %[g], 0", "s_cbranch_scc1 9f",
          "s_sub_u32 %[wc], %[wc], 1", "s_cmp_lg_u32 %[wc], 0", "s_cbranch_scc1 1b",
          "s_mov_b64 %[m], %[k1]", "s_mov_b32 %[wc], 4", "s_branch 1b",
          "9:", "s_waitcnt lgkmcnt(0)"]
    return f"""
// gslcblas dnrm2's ssq recurrence over p[0 .. 16 g) (g <= 8): element e is a
// new running maximum where bit e of (k1:k0) is set, ssq = 1 + (ssq t) t,
// else ssq += t (GSL's operation order; SURVEY.md Appendix A)
__device__ __forceinline__ double kc_nrm2(double acc, unsigned p, unsigned g, unsigned long long k0,
                                          unsigned long long k1) {{
  unsigned long long m, t;
  unsigned wc;
  double tmp;
  asm volatile(
{asm_block(L)}
      : [acc] "+v"(acc), [p] "+v"(p), [g] "+s"(g), [m] "=&s"(m), [t] "=&s"(t), [wc] "=&s"(wc), [tmp] "=&v"(tmp)
      : [k0] "s"(k0), [k1] "s"(k1)
      : "scc", "memory", {CLOBBER});
  return acc;
}}
"""


def emit_lock(desc):
    """Lockstep per-lane chains acc_lane + sum_t w_t m_t (each product
    rounded, then added): w wave-uniform (broadcast LDS reads), m per lane.
    8-element batches, the next batch's loads in flight while the current
    one is multiplied and added (set A: w slots 0-7, m 8-15; set B: w
    16-23, m 24-31)."""

    def load(setb):
        ws, ms = (16, 24) if setb else (0, 8)
        out = []
        for k in range(4):
            if desc:  # element t at byte offset (7 - t) * 8 above the batch base
                o0, o1 = 7 - 2 * k, 6 - 2 * k
                out.append(f"ds_read2_b64 {q(ws // 2 + k)}, %[pw] offset0:{o0} offset1:{o1}")
                out.append(f"ds_read2_b64 {q(ms // 2 + k)}, %[pm] offset0:{o0} offset1:{o1}")
            else:
                out.append(f"ds_read2_b64 {q(ws // 2 + k)}, %[pw] offset0:{2 * k} offset1:{2 * k + 1}")
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
            out.append(f"v_mul_f64 {d(ws + t)}, {d(ws + t)}, {d(ms + t)}")
            for _ in range(per):  # the other set's loads fill this batch's stall slots
                if li < len(loads):
                    out.append(loads[li])
                    li += 1
            out.append(f"v_add_f64 %[acc], %[acc], {d(ws + t)}")
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
// m per lane); the loads run one batch below the last element.
__device__ __forceinline__ double kc_lock_desc(double acc, unsigned pw, unsigned pm, unsigned nb) {{
  asm volatile(
{body}
      : [acc] "+v"(acc), [pw] "+v"(pw), [pm] "+v"(pm), [nb] "+s"(nb)
      :
      : "scc", "memory", {CLOBBER});
  return acc;
}}
"""
    offs = ", ".join(f'[o{t}] "i"({t} * S)' for t in range(8))
    return f"""
// per-lane chain acc + w[0] m[0] + w[1] m[S] + w[2] m[2 S] + ... over 8 nb
// elements (gslcblas dsymv's ascending t2 walk).  pw = LDS byte address of
// w[0] (uniform), pm = per-lane LDS byte address of m[0], S = the m stride
// in bytes; the loads run one batch past the last element.
template <int S>
__device__ __forceinline__ double kc_lock_asc(double acc, unsigned pw, unsigned pm, unsigned nb) {{
  asm volatile(
{body}
      : [acc] "+v"(acc), [pw] "+v"(pw), [pm] "+v"(pm), [nb] "+s"(nb)
      : [s8] "i"(8 * S), {offs}
      : "scc", "memory", {CLOBBER});
  return acc;
}}
"""


def main():
    hdr = f"""// kg_chains.hpp — GENERATED by tools/gen_chains.py; do not edit.
//
// Ordered FP64 chains of the GSL-order tridiagonalisation as hand-scheduled
// gfx950 assembly (see the generator's docstring for why and how).  Every
// chain keeps the reference's operation order; +,* are IEEE correctly
// rounded on gfx950, so the results equal the oracle's bit for bit.
#pragma once
namespace kg {{
namespace chains {{
{emit_add()}{emit_add_desc()}{emit_nrm2()}{emit_lock(True)}{emit_lock(False)}
}}  // namespace chains
}}  // namespace kg
"""
    with open(OUT, "w") as f:
        f.write(hdr)
    print("wrote", OUT)


if __name__ == "__main__":
    main()
