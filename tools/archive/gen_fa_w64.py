#!/usr/bin/env python3
"""Generator of the hand-scheduled K/V loop of the one-wave-per-SIMD flash-attention forward
(``fa_fwd_w64a_kernel`` in llmctl/ops/csrc/flash_attn_fwd.hip): writes
llmctl/ops/csrc/fa_w64_asm.inc, one inline-asm program per wave that owns its registers by literal
name (hipcc pads nothing inside an asm string and cannot address the sub-registers of an operand,
so the whole loop is one statement: guide §5.7).

Structure (guide App. B 'one wave per SIMD' attention; MI355X_MICROARCH issue prices).  A wave
holds two 32-row query blocks A | B; per 64-key tile t two phases of 32 v_mfma_f32_32x32x16_bf16:
    phase 1(t) : S_A(t), S_B(t) = K_t Q^T           | finish softmax B(t-1) | V_{t-1} tr-reads | DMA t+2
    --- barrier: tile t+1 landed, every wave past phase 1(t) ---
    phase 2(t) : O_A, O_B += V_{t-1}^T P(t-1)      | start softmax A(t), B(t) (max, rescale decision),
                                                     finish softmax A(t)   | K_{t+1} b128-reads
so each phase reads one operand's fragments for the other phase (K into a[192:255], V^T into
v[96:159]) and the 128 KiB of LDS fragment traffic a workgroup moves per tile is spread over the
whole tile instead of one phase (a design reading both in one phase measured its LDS reads at
~600 cycles per phase: tools/attn_fwd_ab.py --stamps, profiles/attn_fwd_w64_r5.txt).  Every MFMA
gap carries <= 24 issue cycles of fillers (v_exp 8, other VALU / SALU 4, a DMA piece 12); block
B's exps precede the QK^T MFMAs that overwrite S_B (deadlines), block A's P^T writes follow the PV
MFMAs that read the previous P^T.  Only a wave's last tile (its causal diagonal / the sequence
end) runs the masked softmax.

Register map (per wave):
    a[0:63] O_A (d block d at a[16d:+15])    a[64:127] O_B    a[128:159] Q_A    a[160:191] Q_B
    a[192:255] K_t fragments (kb, ks) at a[192 + 4 (8 kb + ks)]
    v[0:31] S_A (kb at v[16 kb:+15])   v[32:63] S_B   v[64:79] P_A   v[80:95] P_B (dword e/2)
    v[96:159] V^T fragments (kb, st, d) at v[96 + 4 (8 kb + 4 st + d)]
    v[160:175] K / V fragment addresses, then softmax temporaries, m / l / alpha / -m per block
    s[48:99] descriptors, tile counter, slot offsets, grow masks, DMA cursors (+ stamps)

    python tools/gen_fa_w64.py        # rewrites llmctl/ops/csrc/fa_w64_asm.inc
"""
import os

KB = 64
ROWB = 256            # bytes per K/V row (HD 128 bf16)
TILE = KB * ROWB      # 16 KiB: one K or V tile image
SLOT = 2 * TILE       # K | V
GAP_CYC = 24          # issue cycles hidden per MFMA gap (one wave per SIMD)
GAP_N = 5             # ... and at most this many fillers


# ---- registers
def S(z, e): return 32 * z + e                      # score element e (kb = e // 16, i = e % 16)
def P(z, e2): return 64 + 16 * z + e2               # packed P^T dword (elements 2 e2, 2 e2 + 1)
def O(x, d): return 64 * x + 16 * d                 # AGPR base of O_x d-block
def Q(x, ks): return 128 + 32 * x + 4 * ks          # AGPR base of Q_x k-step
def KF(kb, ks): return 192 + 4 * (8 * kb + ks)      # AGPR base of a K fragment
def VF(kb, st, d): return 96 + 4 * (8 * kb + 4 * st + d)


KADDR = 160                                         # K fragment addresses (ks)
VADDR = 168                                         # V fragment addresses (d, lo / hi)
MX, T, MN, RS, T2, LIM = range(176, 182)
def NM(z): return 182 + z                           # -m_new (0 if -inf): exponent offset
def ALPHA(z): return 184 + z
def M(z): return 186 + 2 * z
def L(z): return 187 + 2 * z
RT = 190            # rescale temporaries (4)
VNINF = 194         # -inf (v_cndmask may read one SGPR: its mask)
NVREG = VNINF + 1

# ---- SGPRs
SK, SV, SQ = 48, 52, 56           # buffer descriptors (K, V, Q / O), s[60:63] LSE
ST, SSLK, SSLV, SKV0 = 64, 65, 66, 67
def SG(z): return 68 + 2 * z      # grow mask of block z (64-bit)
SKC, SVC = 72, 74                 # K / V DMA cursors (64-bit)
SIK, STMP, STMP2, SM0, SNINF = 76, 77, 78, 80, 81
SCMP = (82, 84)                   # compare masks (64-bit), alternating
STMP3 = 86


def vr(b, n):
    return f"v[{b}:{b + n - 1}]"


def ar(b, n):
    return f"a[{b}:{b + n - 1}]"


class Item:
    """One filler instruction (or an indivisible group, lines joined by newlines)."""

    def __init__(self, text, cost, deps, deadline=None, not_before=0):
        self.text, self.cost, self.deps = text, cost, list(deps)
        self.deadline = deadline        # must be issued before MFMA slot `deadline`
        self.not_before = not_before    # may be issued only after MFMA slot `not_before - 1`


class Stream:
    """Dependency-ordered fillers; deps = (item index, wait states between) pairs."""

    def __init__(self):
        self.items = []

    def add(self, text, cost=4, deps=(), deadline=None, not_before=0):
        self.items.append(Item(text, cost, deps, deadline, not_before))
        return len(self.items) - 1

    def extend(self, other):
        base = len(self.items)
        for it in other.items:
            self.items.append(Item(it.text, it.cost, [(d + base, w) for d, w in it.deps], it.deadline, it.not_before))


class Emitter:
    def __init__(self, stamps=False):
        self.stamps = stamps
        self.lines = []
        self.pos = 0          # issue position: each instruction 1 wait state, s_nop N N + 1

    def emit(self, text, ws=1):
        for line in text.split("\n"):
            self.lines.append(line)
            self.pos += ws

    def label(self, name):
        self.lines.append(f"{name}:")

    def stamp(self, k):
        """Diagnostic build: s_memtime; cycles since the previous stamp added to accumulator k."""
        if not self.stamps:
            return
        for t in ("s_memtime s[88:89]", "s_waitcnt lgkmcnt(0)", "s_sub_u32 s90, s88, s87",
                  f"s_add_u32 s{91 + k}, s{91 + k}, s90", "s_mov_b32 s87, s88"):
            self.emit(t)

    def nop_until(self, need_pos):
        gap = need_pos - self.pos
        while gap > 0:
            k = min(gap, 8)
            self.emit(f"s_nop {k - 1}", k)
            gap -= k


# ---- softmax streams ---------------------------------------------------------------------------
def start_softmax(st, z, masked, c="%[c]"):
    """Mask (last tile), row max, rescale decision, m_new / -m_new / alpha of block z's S^T."""
    def a(text, cost=4, deps=()):
        return st.add(text, cost, deps)

    first = []
    if masked:
        # key kv0 + idx visible iff idx <= lim = key_hi - kv0 - 4h; two mask pairs alternate so each
        # v_cndmask sits two instructions after its v_cmp (VALU SGPR write -> lane-mask read)
        i_lim = a(f"v_subrev_u32_e32 v{LIM}, s{SKV0}, %[khi{z}]")
        cmps = []

        def cnd(e):
            pr = SCMP[e % 2]
            return a(f"v_cndmask_b32_e64 v{S(z, e)}, v{VNINF}, v{S(z, e)}, s[{pr}:{pr + 1}]", 4, [(cmps[e], 2)])

        for e in range(32):
            kb, i = divmod(e, 16)
            idx = kb * 32 + (i & 3) + 8 * (i >> 2)
            pr = SCMP[e % 2]
            cmps.append(a(f"v_cmp_ge_i32_e64 s[{pr}:{pr + 1}], v{LIM}, {idx}", 4, [(i_lim, 0)]))
            if e >= 1:
                first.append(cnd(e - 1))
        first.append(cnd(31))
    # two independent max chains (MX, T), no back-to-back dependent VALU
    ia = a(f"v_max3_f32 v{MX}, v{S(z, 0)}, v{S(z, 1)}, v{S(z, 2)}", 4, [(x, 0) for x in first])
    ib = a(f"v_max3_f32 v{T}, v{S(z, 3)}, v{S(z, 4)}, v{S(z, 5)}", 4, [(x, 0) for x in first])
    for n, j in enumerate(range(6, 32, 2)):
        if n % 2 == 0:
            ia = a(f"v_max3_f32 v{MX}, v{MX}, v{S(z, j)}, v{S(z, j + 1)}", 4, [(ia, 0)])
        else:
            ib = a(f"v_max3_f32 v{T}, v{T}, v{S(z, j)}, v{S(z, j + 1)}", 4, [(ib, 0)])
    i = a(f"v_max_f32_e32 v{MX}, v{MX}, v{T}", 4, [(ia, 0), (ib, 0)])
    i_mov = a(f"v_mov_b32_e32 v{T}, v{MX}", 4, [(i, 0)])
    i = a(f"v_permlane32_swap_b32_e32 v{MX}, v{T}", 4, [(i_mov, 2)])
    i = a(f"v_max_f32_e32 v{MX}, v{MX}, v{T}", 4, [(i, 0)])
    i_mul = a(f"v_mul_f32_e32 v{MX}, {c}, v{MX}", 4, [(i, 0)])
    # deferred rescale headroom 16 (log2): p <= 2^16 stays exact in fp32 / bf16 (only the exponent
    # grows); a wave rescales when ANY of its 32 rows grows, so 8 triggered ~1 rescale per tile on
    # wide score ranges (tools/attn_fwd_ab.py --qscale 6: 852 cycles per tile; the model step: +20 %)
    i_th = a(f"v_add_f32_e32 v{T}, 0x41800000, v{M(z)}", 4, [(i, 0)])
    i_cmp = a(f"v_cmp_gt_f32_e32 vcc, v{MX}, v{T}", 4, [(i_mul, 0), (i_th, 0)])
    # one item: nothing (a DMA piece's SALU add) may clobber SCC between the two
    i_cs = a(f"s_cmp_lg_u64 vcc, 0\ns_cselect_b64 s[{SG(z)}:{SG(z) + 1}], -1, 0", 8, [(i_cmp, 1)])
    i_mx = a(f"v_max_f32_e32 v{T}, v{M(z)}, v{MX}", 4, [(i_cmp, 0)])
    i_mn = a(f"v_cndmask_b32_e64 v{MN}, v{M(z)}, v{T}, s[{SG(z)}:{SG(z) + 1}]", 4, [(i_cs, 1), (i_mx, 0)])
    # the O rescale is needed only if some row already holds mass (l > 0): not on a block's first
    # tile, where every growing row's max moves up from -inf over an O of zeros
    i_l = a(f"v_cmp_lt_f32_e32 vcc, 0, v{L(z)}", 4, [(i_mn, 0)])
    a(f"s_and_b64 s[{SG(z)}:{SG(z) + 1}], s[{SG(z)}:{SG(z) + 1}], vcc", 4, [(i_l, 1)])
    i_ne = a(f"v_cmp_neq_f32_e64 s[{SCMP[0]}:{SCMP[0] + 1}], s{SNINF}, v{MN}", 4, [(i_mn, 0)])
    i_nm = a(f"v_cndmask_b32_e64 v{NM(z)}, 0, -v{MN}, s[{SCMP[0]}:{SCMP[0] + 1}]", 4, [(i_ne, 2)])
    i_t2 = a(f"v_add_f32_e32 v{T2}, v{M(z)}, v{NM(z)}", 4, [(i_nm, 0)])
    a(f"v_exp_f32_e32 v{ALPHA(z)}, v{T2}", 8, [(i_t2, 0)])
    a(f"v_mov_b32_e32 v{M(z)}, v{MN}", 4, [(i_t2, 0)])


def finish_softmax(st, z, deadlines=None, cvt_not_before=0, c="%[c]"):
    """P^T = 2^(S c - m) of block z (in place, then packed), row sums, l = l alpha + rowsum.
    deadlines(e): MFMA slot before which every read of element e must be issued."""
    def a(text, cost=4, deps=(), e=None, nb=0):
        dl = deadlines(e) if (deadlines and e is not None) else None
        return st.add(text, cost, deps, dl, nb)

    exps = {}
    acc = {0: None, 1: None}   # row sums of the even / odd elements (RS, T2): independent chains

    def rowsum(e):
        r = RS if e % 2 == 0 else T2
        if e < 2:
            return
        if e in (2, 3):
            acc[e % 2] = a(f"v_add_f32_e32 v{r}, v{S(z, e - 2)}, v{S(z, e)}", 4, [(exps[e - 2], 1), (exps[e], 1)], e=e)
        else:
            acc[e % 2] = a(f"v_add_f32_e32 v{r}, v{S(z, e)}, v{r}", 4, [(exps[e], 1), (acc[e % 2], 0)], e=e)

    def cvt(e):  # P^T dword of elements (e - 1, e), e odd
        a(f"v_cvt_pk_bf16_f32 v{P(z, e // 2)}, v{S(z, e - 1)}, v{S(z, e)}", 4, [(exps[e - 1], 1), (exps[e], 1)],
          e=e, nb=cvt_not_before)

    for p2 in range(16):
        e0, e1 = 2 * p2, 2 * p2 + 1
        f0 = a(f"v_fma_f32 v{S(z, e0)}, v{S(z, e0)}, {c}, v{NM(z)}", 4, (), e=e0)
        f1 = a(f"v_fma_f32 v{S(z, e1)}, v{S(z, e1)}, {c}, v{NM(z)}", 4, (), e=e1)
        exps[e0] = a(f"v_exp_f32_e32 v{S(z, e0)}, v{S(z, e0)}", 8, [(f0, 0)], e=e0)
        exps[e1] = a(f"v_exp_f32_e32 v{S(z, e1)}, v{S(z, e1)}", 8, [(f1, 0)], e=e1)
        if p2 >= 1:  # the previous pair: its exps are >= 2 items back
            rowsum(e0 - 2)
            rowsum(e1 - 2)
            if not cvt_not_before:
                cvt(e1 - 2)
    rowsum(30)
    rowsum(31)
    if cvt_not_before:  # the packs wait for the MFMAs that read the previous P^T: all at the end
        for e in range(1, 32, 2):
            cvt(e)
    else:
        cvt(31)
    i_rs = a(f"v_add_f32_e32 v{RS}, v{RS}, v{T2}", 4, [(acc[0], 0), (acc[1], 0)])
    state = {"rs": i_rs}
    i_mv = a(f"v_mov_b32_e32 v{T}, v{RS}", 4, [(state["rs"], 0)])
    i_sw = a(f"v_permlane32_swap_b32_e32 v{RS}, v{T}", 4, [(i_mv, 2)])
    i_ad = a(f"v_add_f32_e32 v{RS}, v{RS}, v{T}", 4, [(i_sw, 0)])
    a(f"v_fma_f32 v{L(z)}, v{L(z)}, v{ALPHA(z)}, v{RS}", 4, [(i_ad, 0)])


# ---- fragment reads, DMA ------------------------------------------------------------------------
def v_reads(st):
    """V^T fragments of the tile in slot SSLV (+ TILE) into VF: 2 ds_read_b64_tr_b16 each."""
    for d in range(4):
        st.add(f"v_add_u32_e32 v{VADDR + 2 * d}, s{SSLV}, %[va{2 * d}]", 4)
        st.add(f"v_add_u32_e32 v{VADDR + 2 * d + 1}, s{SSLV}, %[va{2 * d + 1}]", 4)
    for kb in range(2):
        for s_ in range(2):
            for d in range(4):
                off = (kb * 32 + 16 * s_) * ROWB
                vf = VF(kb, s_, d)
                st.add(f"ds_read_b64_tr_b16 {vr(vf, 2)}, v{VADDR + 2 * d} offset:{off}", 3)
                st.add(f"ds_read_b64_tr_b16 {vr(vf + 2, 2)}, v{VADDR + 2 * d + 1} offset:{off}", 3)


def k_reads(st):
    """K fragments of the tile in slot SSLK into KF (AGPRs): one ds_read_b128 each."""
    for ks in range(8):
        st.add(f"v_add_u32_e32 v{KADDR + ks}, s{SSLK}, %[ka{ks}]", 4)
    for kb in range(2):
        for ks in range(8):
            st.add(f"ds_read_b128 {ar(KF(kb, ks), 4)}, v{KADDR + ks} offset:{kb * 32 * ROWB}", 3)


def dma_items(st):
    """The 8 LDS-DMA pieces of the tile at the cursors (key index s76) into the slot whose M0 base
    is s80; keys >= S (whole dummy tiles past the end included) are outside the descriptors'
    record counts: no LDS write.  Advances the cursors."""
    st.add("\n".join([
        f"s_sub_i32 s{STMP}, %[S], s{SIK}",
        f"s_min_i32 s{STMP}, s{STMP}, {KB}",
        f"s_add_i32 s{STMP2}, s{STMP}, -1",
        f"s_mul_i32 s{STMP2 + 1}, s{STMP2}, %[kss2]",
        f"s_add_i32 s{STMP2 + 1}, s{STMP2 + 1}, {ROWB}",
        f"s_mul_i32 s{STMP3}, s{STMP2}, %[vss2]",
        f"s_add_i32 s{STMP3}, s{STMP3}, {ROWB}",
        f"s_cmp_gt_i32 s{STMP}, 0",            # SALU adds clobber SCC: compare right before its uses
        f"s_cselect_b32 s{SK + 2}, s{STMP2 + 1}, 0",
        f"s_cselect_b32 s{SV + 2}, s{STMP3}, 0",
        f"s_mov_b32 s{SK}, s{SKC}",
        f"s_and_b32 s{SK + 1}, s{SKC + 1}, 0xffff",
        f"s_mov_b32 s{SV}, s{SVC}",
        f"s_and_b32 s{SV + 1}, s{SVC + 1}, 0xffff",
        f"s_add_u32 s{SKC}, s{SKC}, %[kstep]", f"s_addc_u32 s{SKC + 1}, s{SKC + 1}, 0",
        f"s_add_u32 s{SVC}, s{SVC}, %[vstep]", f"s_addc_u32 s{SVC + 1}, s{SVC + 1}, 0",
        f"s_add_i32 s{SIK}, s{SIK}, {KB}"]), 16)
    for i in range(4):
        st.add(f"s_add_u32 m0, s{SM0}, {i * 4096}\ns_nop 0\nbuffer_load_dwordx4 %[vk{i}], s[{SK}:{SK + 3}], 0 offen lds", 12)
        st.add(f"s_add_u32 m0, s{SM0}, {TILE + i * 4096}\ns_nop 0\nbuffer_load_dwordx4 %[vv{i}], s[{SV}:{SV + 3}], 0 offen lds", 12)


def dma_now(em):
    st = Stream()
    dma_items(st)
    for it in st.items:
        em.emit(it.text)


# ---- MFMA lists ---------------------------------------------------------------------------------
def qk_list():
    """S_A (kb 0, 1) then S_B (kb 0, 1): 4 x 8 MFMAs chaining over the 8 k-steps."""
    out = []
    for x in range(2):
        for kb in range(2):
            for ks in range(8):
                src_c = "0" if ks == 0 else vr(S(x, 16 * kb), 16)
                out.append(f"v_mfma_f32_32x32x16_bf16 {vr(S(x, 16 * kb), 16)}, {ar(KF(kb, ks), 4)}, {ar(Q(x, ks), 4)}, {src_c}")
    return out


def pv_list():
    """O_A then O_B += V^T P^T: per block (kb, st) x 4 d blocks."""
    out = []
    for x in range(2):
        for kb in range(2):
            for s_ in range(2):
                for d in range(4):
                    out.append(f"v_mfma_f32_32x32x16_bf16 {ar(O(x, d), 16)}, {vr(VF(kb, s_, d), 4)}, "
                               f"{vr(P(x, 8 * kb + 4 * s_), 4)}, {ar(O(x, d), 16)}")
    return out


def phase(em, mfmas, streams):
    """MFMAs with the streams' fillers in their gaps, round-robin over the streams (each keeps its own
    order); the per-gap issue budget is the phase's filler cost spread evenly (>= GAP_CYC), hazard
    wait states padded, deadlines forced, not-before slots respected; leftovers after the last MFMA."""
    streams = [s_ for s_ in (streams or []) if s_ is not None and s_.items]
    total = sum(it.cost for s_ in streams for it in s_.items)
    budget = max(GAP_CYC, -(-total // max(len(mfmas), 1)) + 2)
    cur = [0] * len(streams)
    pos_of = [dict() for _ in streams]

    def need(k, it):
        return max([pos_of[k][d] + ws for d, ws in it.deps], default=0)

    def put(k):
        it = streams[k].items[cur[k]]
        em.nop_until(need(k, it))
        em.emit(it.text)
        pos_of[k][cur[k]] = em.pos
        cur[k] += 1

    for j, m in enumerate(mfmas):
        for k, s_ in enumerate(streams):  # items due before MFMA j
            due = [n for n in range(cur[k], len(s_.items)) if s_.items[n].deadline is not None and s_.items[n].deadline <= j]
            while due and cur[k] <= due[-1]:
                put(k)
        em.emit(m)
        cyc = 0
        progress = True
        while progress:
            progress = False
            for k, s_ in enumerate(streams):
                if cur[k] >= len(s_.items):
                    continue
                it = s_.items[cur[k]]
                if it.not_before > j:
                    continue
                cost = it.cost + 4 * max(0, need(k, it) - em.pos)
                if cyc > 0 and cyc + cost > budget:
                    continue
                put(k)
                cyc += cost
                progress = True
    for k, s_ in enumerate(streams):
        while cur[k] < len(s_.items):
            put(k)


def rescale(em, z, label):
    """O_z *= alpha_z when the block's max moved (grow mask); branch around otherwise."""
    em.emit(f"s_cmp_lg_u64 s[{SG(z)}:{SG(z) + 1}], 0")
    em.emit(f"s_cbranch_scc0 {label}")
    em.emit("s_nop 7")   # the PV MFMAs' results -> v_accvgpr_read (8-pass XDL write)
    em.emit("s_nop 7")
    em.emit("s_nop 3")
    for base in range(0, 64, 4):
        for k in range(4):
            em.emit(f"v_accvgpr_read_b32 v{RT + k}, a{64 * z + base + k}")
        em.emit("s_nop 1")
        for k in range(4):
            em.emit(f"v_mul_f32_e32 v{RT + k}, v{ALPHA(z)}, v{RT + k}")
        em.emit("s_nop 1")
        for k in range(4):
            em.emit(f"v_accvgpr_write_b32 a{64 * z + base + k}, v{RT + k}")
    em.emit("s_nop 3")
    em.label(label)


def sync(em):
    """Tile j = t + 1's pieces landed (tile j + 1's 8 may fly), barrier (every wave past the
    previous phase); K slot offset of tile j."""
    em.emit("s_waitcnt vmcnt(8)")
    em.emit("s_barrier")
    em.emit(f"s_add_i32 s{STMP}, s{ST}, 1")
    em.emit(f"s_and_b32 s{STMP}, s{STMP}, 3")
    em.emit(f"s_lshl_b32 s{SSLK}, s{STMP}, 15")                 # K_{t+1} slot


def iter_start(em):
    """Tile t: V_{t-1} slot offset, kv0, M0 base of tile t + 2's slot; K_t fragments landed."""
    em.emit(f"s_add_i32 s{STMP}, s{ST}, 3")
    em.emit(f"s_and_b32 s{STMP}, s{STMP}, 3")
    em.emit(f"s_lshl_b32 s{SSLV}, s{STMP}, 15")
    em.emit(f"s_add_i32 s{SSLV}, s{SSLV}, {TILE}")              # V_{t-1}
    em.emit(f"s_lshl_b32 s{SKV0}, s{ST}, 6")                   # kv0 = 64 t
    em.emit(f"s_add_i32 s{STMP}, s{ST}, 2")
    em.emit(f"s_and_b32 s{STMP}, s{STMP}, 3")
    em.emit(f"s_lshl_b32 s{STMP}, s{STMP}, 15")
    em.emit(f"s_add_u32 s{SM0}, %[ldsdma], s{STMP}")           # tile t + 2's slot (+ wave * 1 KiB)
    em.emit("s_waitcnt lgkmcnt(0)")


def b_deadline(e):
    # QK MFMAs: S_A kb0 0-7, S_A kb1 8-15, S_B kb0 16-23, S_B kb1 24-31
    return 16 if e < 16 else 24


def phase1(em, qk=True):
    sm, rd = Stream(), Stream()
    if EXP != "nosm":
        finish_softmax(sm, 1, deadlines=b_deadline if qk else None)
    if EXP != "noread":
        v_reads(rd)
    if EXP != "nodma":
        dma_items(rd)
    phase(em, qk_list() if qk else [], [sm, rd])


def phase2(em, masked=False, pv=True, softmax=True):
    em.emit("s_waitcnt lgkmcnt(0)")   # V fragments landed
    em.emit("s_nop 7")                # phase 1's QK^T results -> the max VALU (8-pass XDL write)
    em.emit("s_nop 7")
    sm, rd = Stream(), Stream()
    if softmax and EXP != "noread":
        k_reads(rd)
    if softmax and EXP != "nosm":
        start_softmax(sm, 0, masked)
        start_softmax(sm, 1, masked)
        # P_A(t) overwrites P_A(t-1): after the 16 PV MFMAs of block A read it
        finish_softmax(sm, 0, cvt_not_before=17 if pv else 0)
    if EXP == "shift":  # (ablation) DMA pieces in phase 2 instead of phase 1
        dma_items(rd)
    phase(em, pv_list() if pv else [], [sm, rd])


def prologue(em):
    em.emit("s_nop 4")
    em.emit(f"s_mov_b32 s{SNINF}, 0xff800000")
    em.emit(f"s_mov_b32 s{SK + 3}, 0x00020000")
    em.emit(f"s_mov_b32 s{SV + 3}, 0x00020000")
    em.emit(f"v_mov_b32_e32 v{VNINF}, s{SNINF}")
    # DMA cursors; tiles 0 and 1 in flight under the Q loads
    em.emit(f"s_mov_b32 s{SKC}, %[kblo]")
    em.emit(f"s_mov_b32 s{SKC + 1}, %[kbhi]")
    em.emit(f"s_mov_b32 s{SVC}, %[vblo]")
    em.emit(f"s_mov_b32 s{SVC + 1}, %[vbhi]")
    em.emit(f"s_mov_b32 s{SIK}, 0")
    em.emit(f"s_mov_b32 s{ST}, 0")
    em.emit(f"s_mov_b32 s{SM0}, %[ldsdma]")
    dma_now(em)
    em.emit(f"s_add_u32 s{SM0}, %[ldsdma], {SLOT}")
    dma_now(em)
    # Q: 8 x 16 B per lane per block, rows >= S read 0 (record bound)
    em.emit(f"s_mov_b32 s{SQ}, %[qlo]")
    em.emit(f"s_and_b32 s{SQ + 1}, %[qhi], 0xffff")
    em.emit(f"s_mov_b32 s{SQ + 2}, %[qnrec]")
    em.emit(f"s_mov_b32 s{SQ + 3}, 0x00020000")
    em.emit("s_nop 0")
    for x, vq in ((0, "%[vqA]"), (1, "%[vqB]")):
        for ks in range(8):
            em.emit(f"buffer_load_dwordx4 {vr(32 * x + 4 * ks, 4)}, {vq}, s[{SQ}:{SQ + 3}], 0 offen offset:{32 * ks}")
    for i in range(128):
        em.emit(f"v_accvgpr_write_b32 a{i}, 0")
    for e2 in range(32):
        em.emit(f"v_mov_b32_e32 v{64 + e2}, 0")         # "P(-1)" = 0
    for z in range(2):
        em.emit(f"v_mov_b32_e32 v{M(z)}, s{SNINF}")
        em.emit(f"v_mov_b32_e32 v{L(z)}, 0")
        em.emit(f"v_mov_b32_e32 v{ALPHA(z)}, 1.0")
        em.emit(f"v_mov_b32_e32 v{NM(z)}, 0")
    em.emit(f"s_mov_b64 s[{SG(0)}:{SG(0) + 1}], 0")
    em.emit(f"s_mov_b64 s[{SG(1)}:{SG(1) + 1}], 0")
    em.emit("s_waitcnt vmcnt(0)")
    for i in range(64):
        em.emit(f"v_accvgpr_write_b32 a{128 + i}, v{i}")
    for e in range(32):
        em.emit(f"v_mov_b32_e32 v{S(1, e)}, s{SNINF}")  # "S_B(-1)" = -inf: the first finish of B is a no-op
    em.emit("s_nop 1")
    # sync(0) and K_0's fragments
    em.emit("s_barrier")
    em.emit(f"s_mov_b32 s{SSLK}, 0")
    st = Stream()
    k_reads(st)
    for it in st.items:
        em.emit(it.text)


def epilogue(em):
    """O / l and the LSE of both blocks, stored before the wave's drain (its stores overlap the
    other waves' last tiles; in-order vmcnt makes the drain's counted waits cover them)."""
    em.emit(f"s_mov_b32 s{SQ}, %[olo]")
    em.emit(f"s_and_b32 s{SQ + 1}, %[ohi], 0xffff")
    em.emit(f"s_mov_b32 s{SQ + 2}, %[onrec]")
    em.emit(f"s_mov_b32 s{SQ + 3}, 0x00020000")
    em.emit("s_mov_b32 s60, %[llo]")
    em.emit("s_and_b32 s61, %[lhi], 0xffff")
    em.emit("s_mov_b32 s62, %[lnrec]")
    em.emit("s_mov_b32 s63, 0x00020000")
    em.emit("s_nop 7")
    em.emit("s_nop 7")
    for z in range(2):
        inv, lse = T, T2
        em.emit(f"v_rcp_f32_e32 v{inv}, v{L(z)}")
        em.emit(f"v_log_f32_e32 v{lse}, v{L(z)}")
        em.emit(f"v_cmp_lt_f32_e32 vcc, 0, v{L(z)}")
        em.emit("s_nop 1")
        em.emit(f"v_cndmask_b32_e32 v{inv}, 0, v{inv}, vcc")
        em.emit(f"v_add_f32_e32 v{lse}, v{M(z)}, v{lse}")
        em.emit(f"v_mul_f32_e32 v{lse}, 0x3f317218, v{lse}")
        em.emit(f"v_cndmask_b32_e32 v{lse}, v{VNINF}, v{lse}, vcc")
        em.emit("s_nop 1")
        em.emit(f"buffer_store_dword v{lse}, %[vl{z}], s[60:63], 0 offen")
        for d in range(4):
            for g in range(4):
                r0 = 8 * ((4 * d + g) % 8)
                for j in range(4):
                    em.emit(f"v_accvgpr_read_b32 v{r0 + j}, a{64 * z + 16 * d + 4 * g + j}")
                em.emit("s_nop 1")
                for j in range(4):
                    em.emit(f"v_mul_f32_e32 v{r0 + j}, v{inv}, v{r0 + j}")
                em.emit(f"v_cvt_pk_bf16_f32 v{r0 + 4}, v{r0}, v{r0 + 1}")
                em.emit(f"v_cvt_pk_bf16_f32 v{r0 + 5}, v{r0 + 2}, v{r0 + 3}")
                em.emit("s_nop 1")
                em.emit(f"buffer_store_dwordx2 v[{r0 + 4}:{r0 + 5}], %[vo{z}], s[{SQ}:{SQ + 3}], 0 offen offset:{d * 64 + g * 16}")
        em.emit("s_nop 1")


SECTIONS = ("prologue", "phase1", "sync", "phase2", "rescale+loop", "last", "tail", "drain", "epilogue")
EXP = ""  # diagnostic ablations of the stamp builds: nosm (no softmax), noread (no fragment reads)


def program(stamps=False, exp=""):
    global EXP
    EXP = exp
    em = Emitter(stamps)
    if stamps:
        for k in range(9):
            em.emit(f"s_mov_b32 s{91 + k}, 0")
        em.emit("s_memtime s[88:89]")
        em.emit("s_waitcnt lgkmcnt(0)")
        em.emit("s_mov_b32 s87, s88")
    prologue(em)
    em.stamp(0)
    em.emit(f"s_cmp_lt_i32 %[tw], 0")
    em.emit("s_cbranch_scc1 L_dead_%=")
    em.emit(f"s_cmp_lt_i32 s{ST}, %[tw]")
    em.emit("s_cbranch_scc0 L_last_%=")
    em.label("L_loop_%=")
    # ---- tiles before the wave's last one
    iter_start(em)
    phase1(em)
    em.stamp(1)
    sync(em)
    em.stamp(2)
    phase2(em)
    em.stamp(3)
    rescale(em, 0, "L_rsal_%=")
    rescale(em, 1, "L_rsbl_%=")
    em.emit(f"s_add_i32 s{ST}, s{ST}, 1")
    em.stamp(4)
    em.emit(f"s_cmp_lt_i32 s{ST}, %[tw]")
    em.emit("s_cbranch_scc1 L_loop_%=")
    em.label("L_last_%=")
    # ---- the last tile (causal diagonal / sequence end): both blocks' softmax masked
    iter_start(em)
    phase1(em)
    sync(em)
    phase2(em, masked=True)
    rescale(em, 0, "L_rsat_%=")
    rescale(em, 1, "L_rsbt_%=")
    em.emit(f"s_add_i32 s{ST}, s{ST}, 1")
    em.stamp(5)
    # ---- tail: finish B(tw), V_tw's fragments, then O += V_tw^T P(tw)
    iter_start(em)
    phase1(em, qk=False)
    sync(em)
    em.emit("s_waitcnt lgkmcnt(0)")
    em.emit("s_nop 1")
    phase(em, pv_list(), [])
    em.emit(f"s_add_i32 s{STMP}, s{ST}, 3")             # tile t + 3 (= tw + 4: past the end, no write)
    em.emit(f"s_and_b32 s{STMP}, s{STMP}, 3")
    em.emit(f"s_lshl_b32 s{STMP}, s{STMP}, 15")
    em.emit(f"s_add_u32 s{SM0}, %[ldsdma], s{STMP}")
    dma_now(em)
    em.emit(f"s_add_i32 s{ST}, s{ST}, 2")
    em.stamp(6)
    epilogue(em)
    em.stamp(8)
    em.emit("s_branch L_drain_%=")
    # ---- waves without rows: the DMA share of tile 2 after sync(0)
    em.label("L_dead_%=")
    em.emit(f"s_add_u32 s{SM0}, %[ldsdma], {2 * SLOT}")
    dma_now(em)
    em.emit(f"s_mov_b32 s{ST}, 1")
    # ---- every wave passes ntiles + 2 barriers (sync 0 .. ntiles + 1) and issues its DMA share of
    #      every tile; sync(j) is followed by tile j + 2's pieces
    em.label("L_drain_%=")
    em.emit(f"s_add_i32 s{STMP}, %[ntiles], 1")
    em.emit(f"s_cmp_le_i32 s{ST}, s{STMP}")
    em.emit("s_cbranch_scc0 L_epi_%=")
    em.label("L_dloop_%=")
    em.emit("s_waitcnt vmcnt(8)")
    em.emit("s_barrier")
    em.emit(f"s_add_i32 s{STMP}, s{ST}, 2")
    em.emit(f"s_and_b32 s{STMP}, s{STMP}, 3")
    em.emit(f"s_lshl_b32 s{STMP}, s{STMP}, 15")
    em.emit(f"s_add_u32 s{SM0}, %[ldsdma], s{STMP}")
    dma_now(em)
    em.emit(f"s_add_i32 s{ST}, s{ST}, 1")
    em.emit(f"s_add_i32 s{STMP}, %[ntiles], 1")
    em.emit(f"s_cmp_le_i32 s{ST}, s{STMP}")
    em.emit("s_cbranch_scc1 L_dloop_%=")
    em.label("L_epi_%=")
    em.stamp(7)
    em.emit("s_waitcnt vmcnt(0)")   # no LDS-DMA may land after the workgroup ends
    if stamps:
        em.emit("s_mov_b32 s56, %[stlo]")
        em.emit("s_and_b32 s57, %[sthi], 0xffff")
        em.emit("s_mov_b32 s58, 0x40000")  # [1024 workgroups][4 waves][16 dwords]: lanes at 0x40000000 drop
        em.emit("s_mov_b32 s59, 0x00020000")
        for k in range(9):
            em.emit(f"v_mov_b32_e32 v{k}, s{91 + k}")
        em.emit("s_nop 1")
        for k in range(9):
            em.emit(f"buffer_store_dword v{k}, %[vst], s[56:59], 0 offen offset:{4 * k}")
        em.emit("s_waitcnt vmcnt(0)")
    return em.lines


def main():
    lines = program()
    variants = [program(stamps=True, exp=e) for e in ("", "nosm", "noread", "nodma")]
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    out = os.path.join(root, "llmctl", "ops", "csrc", "fa_w64_asm.inc")
    n_mfma = sum(1 for l in lines if l.startswith("v_mfma"))

    def macro(name, ls):
        return f"#define {name} \\\n" + " \\\n".join(f'  "{l}\\n"' for l in ls) + "\n"

    with open(out, "w") as f:
        f.write("// GENERATED by tools/gen_fa_w64.py -- do not edit.  K/V loop of fa_fwd_w64a_kernel\n")
        f.write(f"// (one inline-asm program, {len(lines)} lines, {n_mfma} MFMAs); register map in the generator.\n")
        f.write(macro("FA_W64_ASM", lines))
        f.write("// diagnostic build (knob fa_stamp_ptr): per-wave cycle totals of the sections\n// "
                + ", ".join(SECTIONS) + "\n")
        for m, vl in enumerate(variants, 1):
            f.write(macro(f"FA_W64_ASM_S{m}", vl))
        regs = [f'"v{i}"' for i in range(NVREG)] + [f'"a{i}"' for i in range(256)] + \
               [f'"s{i}"' for i in range(SK, 100)] + ['"vcc"', '"scc"', '"m0"', '"memory"']
        f.write("#define FA_W64_CLOBBERS " + ", ".join(regs) + "\n")
    print(f"wrote {out}: {len(lines)} lines, {n_mfma} MFMAs")


if __name__ == "__main__":
    main()
