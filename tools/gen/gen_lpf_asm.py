"""Generate csrc/ssb_lpf_asm.h: the SSB pipeline's three serial roles (DC tracker, low-pass, AGC gain), one 64-sample
chunk each, as hand-scheduled asm blocks.

DC wave (removeDC, ssb_demod_opt.cpp:49-55, and iir2Process's a0 x product): see dc_pair(); two samples per group
of seven instructions (the order-free products and the v - dc / a0 steps packed over sample pairs).

Low-pass wave (iir2Process, ssb_demod_opt.cpp:75-84), per sample in the reference's float order without
contraction (products rounded, adds left to right):
    y = (((a0x + a1 z1) + a2 z2) + (-b1) z1) + (-b2) z2
with a0x from the DC wave, (a1 z1, -b1 z1) and (a2 z2, -b2 z2) as two v_pk_mul_f32 broadcasting z1 / z2, and the
four adds in order.

AGC gain wave (adaptiveAGC, ssb_demod_opt.cpp:101-115), per sample:
    cand = gain * {1 - fast, 1 - slow} + desired * {fast, slow}      (each lane: gain*(1-rate) + desired*rate)
    gain = desired < gain ? cand.x : cand.y
as two v_pk_mul_f32 (the desired product first: it does not wait for the gain), v_cmp, v_pk_add, v_cndmask.

Every output is written in place over its input register, and the carried values are read from the half of the
aligned register pair that holds them (op_sel), so a chunk needs no register moves.  The chunk's 64 samples go
through three rotating 16-register sub-block buffers (v0-15, v16-31, v32-47): sub-block k + 2 is read from LDS
while sub-block k runs, and each wait names exactly the LDS operations still allowed in flight, so the only
exposed LDS latency is the chunk's first read.
Run: python tools/gen/gen_lpf_asm.py > sdr-for-android-lib_amd/csrc/ssb_lpf_asm.h
     python tools/gen/gen_lpf_asm.py --lab > tools/lab/lab_lpf_asm.h   (lab-only variants, not in the product)
"""

BUFS = [0, 16, 32]
P1, P2 = 48, 50   # product registers
T0 = 52           # v[52:53]: the AGC's incoming gain as a register pair


def pair(reg):
    """(aligned pair text, half) of a scalar VGPR"""
    base = reg & ~1
    return f"v[{base}:{base + 1}]", reg & 1


def lpf_sample(x, z1, z2):
    """x: input/output VGPR; z1, z2: (pair text, half) of the previous two outputs"""
    p1, h1 = z1
    p2, h2 = z2
    return [
        f"v_pk_mul_f32 v[{P1}:{P1 + 1}], %[c1], {p1} op_sel:[0,{h1}] op_sel_hi:[1,{h1}]",
        f"v_pk_mul_f32 v[{P2}:{P2 + 1}], %[c2], {p2} op_sel:[0,{h2}] op_sel_hi:[1,{h2}]",
        f"v_add_f32 v{x}, v{x}, v{P1}",
        f"v_add_f32 v{x}, v{x}, v{P2}",
        f"v_add_f32 v{x}, v{x}, v{P1 + 1}",
        f"v_add_f32 v{x}, v{x}, v{P2 + 1}",
    ]


def agc_sample(x, g):
    """x: desired in, gain out; g: the previous gain's VGPR"""
    px, hx = pair(x)
    pg, hg = pair(g)
    return [
        f"v_pk_mul_f32 v[{P2}:{P2 + 1}], %[rates], {px} op_sel:[0,{hx}] op_sel_hi:[1,{hx}]",
        f"v_pk_mul_f32 v[{P1}:{P1 + 1}], %[keep], {pg} op_sel:[0,{hg}] op_sel_hi:[1,{hg}]",
        f"v_cmp_lt_f32 vcc, v{x}, v{g}",
        f"v_pk_add_f32 v[{P1}:{P1 + 1}], v[{P1}:{P1 + 1}], v[{P2}:{P2 + 1}]",
        f"v_cndmask_b32 v{x}, v{P1 + 1}, v{P1}, vcc",
    ]


def dc_pair(x, prev):
    """removeDC (ssb_demod_opt.cpp:49-55) for samples x, x + 1 (x even) and the a0 product of iir2Process:
    dc = alpha dc + (1 - alpha) v, v' = a0 (v - dc).  The (1 - alpha) v products of both samples are one packed
    multiply, the two dc steps run on v48 / v49 (so the pair {dc_x, dc_x+1} is v[48:49]), then v - dc and the a0
    product are one packed op each over the sample pair.  prev: the VGPR holding the dc before sample x."""
    return [
        f"v_pk_mul_f32 v[50:51], %[om2], v[{x}:{x + 1}]",
        f"v_mul_f32 v52, %[alpha], v{prev}",
        f"v_add_f32 v48, v52, v50",
        f"v_mul_f32 v52, %[alpha], v48",
        f"v_add_f32 v49, v52, v51",
        f"v_pk_add_f32 v[{x}:{x + 1}], v[{x}:{x + 1}], v[48:49] neg_lo:[0,1] neg_hi:[0,1]",
        f"v_pk_mul_f32 v[{x}:{x + 1}], %[a02], v[{x}:{x + 1}]",
    ]


def reads(sb, buf):
    return [f"ds_read_b128 v[{buf + 4 * i}:{buf + 4 * i + 3}], %[src] offset:{(16 * sb + 4 * i) * 4}" for i in range(4)]


def writes(sb, buf):
    return [f"ds_write_b128 %[dst], v[{buf + 4 * i}:{buf + 4 * i + 3}] offset:{(16 * sb + 4 * i) * 4}" for i in range(4)]


def chunk(role, lds=True, split=False, il=False):
    """role 'dc', 'lpf' or 'agc'.  split (low-pass, lab): VALU with all 64 lanes on (lanes past the 16 streams compute on whatever their
    registers hold and store nothing), LDS operations with the caller's EXEC (saved in %[sv])"""
    out = []

    def exec_lds(ops):
        return ([f"s_mov_b64 exec, %[sv]"] + ops + ["s_mov_b64 exec, -1"]) if (split and ops) else ops

    if split:
        out += ["s_mov_b64 %[sv], exec"] + ([] if lds else ["s_mov_b64 exec, -1"])
    buf = [BUFS[sb % 3] for sb in range(4)]
    if lds:
        out += exec_lds(reads(0, buf[0]) + reads(1, buf[1]))
    # LGKM operations issued after sub-block sb's reads when sb starts: R1 (4) for sb 0; W(sb-1) + R(sb+1) (8)
    # for sb 1, 2; W2 (4) for sb 3
    waits = {0: 4, 1: 8, 2: 8, 3: 4}
    if role == "lpf":
        prev1, prev2 = ("%[z]", 0), ("%[z]", 1)  # z.x = z1, z.y = z2 of the chunk's first sample
    elif role == "dc":
        out.append("v_mov_b32 v49, %[dc]")  # the incoming dc
    else:
        out.append(f"v_pk_mov_b32 v[{T0}:{T0 + 1}], %[g], %[g] op_sel:[0,0]")  # the incoming gain as a VGPR
        g = T0
    for sb in range(4):
        if lds:
            out.append(f"s_waitcnt lgkmcnt({waits[sb]})")
        b = buf[sb]
        for q in range(16):
            if role == "dc":
                if q % 2 == 0:
                    out += dc_pair(b + q, 49)
            elif role == "lpf":
                out += lpf_sample(b + q, prev1, prev2)
                prev2, prev1 = prev1, pair(b + q)
            else:
                out += agc_sample(b + q, g)
                g = b + q
            if il and lds and q % 4 == 3:  # interleaved: this quad's write and sub-block sb + 2's same quad
                t = q // 4
                out += exec_lds(writes(sb, b)[t:t + 1] + (reads(sb + 2, buf[sb + 2])[t:t + 1] if sb + 2 < 4 else []))
        if lds and not il:
            out += exec_lds(writes(sb, b) + (reads(sb + 2, buf[sb + 2]) if sb + 2 < 4 else []))
    last = buf[3] + 15
    if split:  # the carried state is written on the caller's lanes only
        out.append("s_mov_b64 exec, %[sv]")
    if role == "dc":
        out.append("v_mov_b32 %[dc], v49")
    elif role == "lpf":  # carry (z1, z2) = (y63, y62): one v_pk_mov_b32 from the aligned pair holding both
        out.append(f"v_pk_mov_b32 %[z], v[{last - 1}:{last}], v[{last - 1}:{last}] op_sel:[1,0]")
    else:
        out.append(f"v_pk_mov_b32 %[g], v[{last - 1}:{last}], v[{last - 1}:{last}] op_sel:[1,1]")
    return out


SLOT = 16 * 68 * 4  # bytes per [stream][sample] chunk buffer (PG x ROW floats)


def lpf_loop():
    """The low-pass wave's whole chunk loop (SDRG_LPF_LOOKAHEAD): one s_barrier per iteration, like every other
    role's loop, and chunk c = it - 3 (one iteration behind the DC wave's output, through a 3-slot ring), so the
    next chunk's input is complete while this chunk runs: its first two sub-blocks are read before the barrier
    and stay in flight across it (the barrier waits only for this chunk's output writes).  Sub-block j of chunk
    c lives in buffer (c + j) mod 3; three copies of the chunk body, one per c mod 3.
    Operands: %[z] (+v {z1, z2}), %[abase] / %[ybase] (v: LDS byte address of slot 0 of the input / output ring
    at this stream's row), %[c1], %[c2] (s), %[nit] (s: iterations), %[nch] (s: chunks, all full), temps %[sv]
    (=&s 64-bit), %[it], %[cc], %[r], %[yo] (=&s); clobbers v0-v54, vcc-free."""
    out = []
    u = "%="
    out += [
        "s_mov_b64 %[sv], exec",
        "s_mov_b64 exec, 0xffff",          # the 16 stream lanes
        "s_nop 4",
        f"v_pk_mov_b32 v[46:47], %[z], %[z] op_sel:[1,0]",   # chunk -1's sb3 buffer (2): v47 = z1, v46 = z2
        f"v_pk_mov_b32 v[52:53], %[z], %[z] op_sel:[0,1]",   # the carried {z1, z2} if no chunk runs
        "s_mov_b32 %[it], 0",
        "s_mov_b32 %[cc], -3",
        "s_mov_b32 %[r], 0",               # c mod 3 once c >= 0
        f"L_top_{u}:",
        "s_cmp_lt_i32 %[cc], 0",
        f"s_cbranch_scc1 L_pre_{u}",
        "s_cmp_ge_i32 %[cc], %[nch]",
        f"s_cbranch_scc1 L_drain_{u}",
        # output slot c mod 4
        "s_and_b32 %[yo], %[cc], 3",
        f"s_mul_i32 %[yo], %[yo], {SLOT}",
        "v_add_u32 v54, %[yo], %[ybase]",
        "s_cmp_eq_u32 %[r], 0",
        f"s_cbranch_scc1 L_r0_{u}",
        "s_cmp_eq_u32 %[r], 1",
        f"s_cbranch_scc1 L_r1_{u}",
        f"s_branch L_r2_{u}",
    ]
    for r in range(3):
        out.append(f"L_r{r}_{u}:")
        bufs = [BUFS[(r + j) % 3] for j in range(4)]
        zb = BUFS[(r + 2) % 3]
        prev1, prev2 = pair(zb + 15), pair(zb + 14)
        rd = lambda sb, buf, slot: [f"ds_read_b128 v[{buf + 4 * i}:{buf + 4 * i + 3}], %[abase] offset:{slot * SLOT + (16 * sb + 4 * i) * 4}" for i in range(4)]
        wr = lambda sb, buf: [f"ds_write_b128 v54, v[{buf + 4 * i}:{buf + 4 * i + 3}] offset:{(16 * sb + 4 * i) * 4}" for i in range(4)]
        waits = {0: 4, 1: 8, 2: 8, 3: 4}
        for sb in range(4):
            out.append(f"s_waitcnt lgkmcnt({waits[sb]})")
            b = bufs[sb]
            for q in range(16):
                out += lpf_sample(b + q, prev1, prev2)
                prev2, prev1 = prev1, pair(b + q)
            out += wr(sb, b)
            if sb + 2 < 4:
                out += rd(sb + 2, bufs[sb + 2], r)
        last = bufs[3] + 15
        out.append(f"v_pk_mov_b32 v[52:53], v[{last - 1}:{last}], v[{last - 1}:{last}] op_sel:[1,0]")
        # prefetch the next chunk's sub-blocks 0 and 1 (slot (r + 1) mod 3, buffers (r + 1), (r + 2) mod 3)
        out += ["s_add_u32 %[yo], %[cc], 1", "s_cmp_ge_i32 %[yo], %[nch]", f"s_cbranch_scc1 L_drain_{u}"]
        nr = (r + 1) % 3
        out += rd(0, BUFS[nr], nr) + rd(1, BUFS[(nr + 1) % 3], nr)
        out.append(f"s_branch L_bar8_{u}")
    out += [
        f"L_pre_{u}:",                      # c < 0: chunk 0's sub-blocks 0, 1 once c == -1 (chunk 0 is complete)
        "s_cmp_lg_i32 %[cc], -1",
        f"s_cbranch_scc1 L_drain_{u}",
        "s_cmp_le_i32 %[nch], 0",
        f"s_cbranch_scc1 L_drain_{u}",
    ]
    out += [f"ds_read_b128 v[{BUFS[0] + 4 * i}:{BUFS[0] + 4 * i + 3}], %[abase] offset:{(4 * i) * 4}" for i in range(4)]
    out += [f"ds_read_b128 v[{BUFS[1] + 4 * i}:{BUFS[1] + 4 * i + 3}], %[abase] offset:{(16 + 4 * i) * 4}" for i in range(4)]
    out += [
        f"L_bar8_{u}:",
        "s_waitcnt lgkmcnt(8)",            # this chunk's output writes done; the 8 prefetch reads may fly on
        f"s_branch L_bar_{u}",
        f"L_drain_{u}:",
        "s_waitcnt lgkmcnt(0)",
        f"L_bar_{u}:",
        "s_barrier",
        # next iteration: it + 1, c + 1, r = c mod 3 (for c >= 0)
        "s_add_u32 %[it], %[it], 1",
        "s_add_i32 %[cc], %[cc], 1",
        "s_cmp_le_i32 %[cc], 0",
        f"s_cbranch_scc1 L_next_{u}",      # c <= 0 after the increment: r stays 0
        "s_add_u32 %[r], %[r], 1",
        "s_cmp_eq_u32 %[r], 3",
        "s_cselect_b32 %[r], 0, %[r]",
        f"L_next_{u}:",
        "s_cmp_lt_u32 %[it], %[nit]",
        f"s_cbranch_scc1 L_top_{u}",
        "s_mov_b64 exec, %[sv]",
        "s_nop 4",
        "v_pk_mov_b32 %[z], v[52:53], v[52:53] op_sel:[0,1]",
    ]
    return out


def lpf_loop_interleaved(copies=False, split=False):
    """lpf_loop() with the LDS traffic spread through the VALU stream: sub-blocks are numbered g = 4c + sb across
    chunks and live in buffer g mod 3; while sub-block g runs, after each 4-sample quad t its output quad is written
    and quad t of sub-block g + 2 is read (for sb = 2, 3 that is the next chunk's sub-block 0, 1, complete in its
    ring slot).  So at the barrier only the chunk's last write is outstanding (lgkmcnt(1)), and the first two
    sub-blocks of the next chunk are already in registers.  The last chunk's reads of a next chunk fetch a stale
    ring slot and are never used; the block drains them (lgkmcnt(0)) before it ends.
    Lab forms (--lab, not in the product): copies, all 64 lanes with lane l running stream l mod 16 (four copies: a
    dependent chain issues faster on a full EXEC mask, and the copies write the same values to the same LDS
    addresses); split, the chain's VALU on all 64 lanes (lanes 16-63 compute on whatever they hold and store nothing),
    each quad's LDS write and read on the 16 stream lanes (EXEC switched by SALU around the pair)."""
    assert not (copies and split)
    out = []
    u = "%="
    lanes = ["s_mov_b64 exec, -1"] if copies or split else ["s_mov_b64 exec, 0xffff"]
    out += ["s_mov_b64 %[sv], exec"] + lanes + [
        "s_nop 4",
        "v_pk_mov_b32 v[46:47], %[z], %[z] op_sel:[1,0]",
        "v_pk_mov_b32 v[52:53], %[z], %[z] op_sel:[0,1]",
        "s_mov_b32 %[it], 0",
        "s_mov_b32 %[cc], -3",
        "s_mov_b32 %[r], 0",
        f"L_top_{u}:",
        "s_cmp_lt_i32 %[cc], 0",
        f"s_cbranch_scc1 L_pre_{u}",
        "s_cmp_ge_i32 %[cc], %[nch]",
        f"s_cbranch_scc1 L_drain_{u}",
        "s_and_b32 %[yo], %[cc], 3",
        f"s_mul_i32 %[yo], %[yo], {SLOT}",
        "v_add_u32 v54, %[yo], %[ybase]",
        "s_cmp_eq_u32 %[r], 0",
        f"s_cbranch_scc1 L_r0_{u}",
        "s_cmp_eq_u32 %[r], 1",
        f"s_cbranch_scc1 L_r1_{u}",
        f"s_branch L_r2_{u}",
    ]
    for r in range(3):
        out.append(f"L_r{r}_{u}:")
        zb = BUFS[(r + 2) % 3]
        prev1, prev2 = pair(zb + 15), pair(zb + 14)
        for sb in range(4):
            out.append(f"s_waitcnt lgkmcnt({4 if sb == 0 else 8})")
            b = BUFS[(r + sb) % 3]
            rb = BUFS[(r + sb + 2) % 3]                      # buffer of sub-block g + 2
            rslot, rsb = (r, sb + 2) if sb < 2 else ((r + 1) % 3, sb - 2)
            for q in range(16):
                out += lpf_sample(b + q, prev1, prev2)
                prev2, prev1 = prev1, pair(b + q)
                if q % 4 == 3:
                    t = q // 4
                    if split:
                        out.append("s_mov_b64 exec, 0xffff")
                    out.append(f"ds_write_b128 v54, v[{b + 4 * t}:{b + 4 * t + 3}] offset:{(16 * sb + 4 * t) * 4}")
                    out.append(f"ds_read_b128 v[{rb + 4 * t}:{rb + 4 * t + 3}], %[abase] offset:{rslot * SLOT + (16 * rsb + 4 * t) * 4}")
                    if split:
                        out.append("s_mov_b64 exec, -1")
        last = BUFS[(r + 3) % 3] + 15
        out.append(f"v_pk_mov_b32 v[52:53], v[{last - 1}:{last}], v[{last - 1}:{last}] op_sel:[1,0]")
        out.append(f"s_branch L_bar1_{u}")
    out += [
        f"L_pre_{u}:",                      # c < 0: chunk 0's sub-blocks 0, 1 once c == -1 (chunk 0 is complete)
        "s_cmp_lg_i32 %[cc], -1",
        f"s_cbranch_scc1 L_drain_{u}",
        "s_cmp_le_i32 %[nch], 0",
        f"s_cbranch_scc1 L_drain_{u}",
    ]
    out += ["s_mov_b64 exec, 0xffff"] if split else []
    out += [f"ds_read_b128 v[{BUFS[0] + 4 * i}:{BUFS[0] + 4 * i + 3}], %[abase] offset:{(4 * i) * 4}" for i in range(4)]
    out += [f"ds_read_b128 v[{BUFS[1] + 4 * i}:{BUFS[1] + 4 * i + 3}], %[abase] offset:{(16 + 4 * i) * 4}" for i in range(4)]
    out += ["s_mov_b64 exec, -1"] if split else []
    out += [
        f"s_branch L_bar_{u}",
        f"L_bar1_{u}:",
        "s_waitcnt lgkmcnt(1)",             # this chunk's writes done; the last read of the next chunk may fly on
        f"s_branch L_bar_{u}",
        f"L_drain_{u}:",
        "s_waitcnt lgkmcnt(0)",
        f"L_bar_{u}:",
        "s_barrier",
        "s_add_u32 %[it], %[it], 1",
        "s_add_i32 %[cc], %[cc], 1",
        "s_cmp_le_i32 %[cc], 0",
        f"s_cbranch_scc1 L_next_{u}",
        "s_add_u32 %[r], %[r], 1",
        "s_cmp_eq_u32 %[r], 3",
        "s_cselect_b32 %[r], 0, %[r]",
        f"L_next_{u}:",
        "s_cmp_lt_u32 %[it], %[nit]",
        f"s_cbranch_scc1 L_top_{u}",
        "s_waitcnt lgkmcnt(0)",             # the last chunk's reads of a next chunk that does not exist
        "s_mov_b64 exec, %[sv]",
        "s_nop 4",
        "v_pk_mov_b32 %[z], v[52:53], v[52:53] op_sel:[0,1]",
    ]
    return out


def emit(name, lines):
    print(f"#define {name} \\")
    for l in lines:
        print(f'    "{l}\\n" \\')
    print('    ""')


def main():
    print("// Generated by tools/gen/gen_lpf_asm.py -- do not edit.  The SSB pipeline's DC, low-pass and AGC waves, one")
    print("// 64-sample chunk each; see the generator for the schedule.  Operands: %[src] / %[dst] (v, LDS byte addresses of the")
    print("// stream's input / output rows); low-pass: %[z] (+v, {z1, z2}), %[c1] = {a1, -b1}, %[c2] = {a2, -b2} (s);")
    print("// AGC: %[g] (+v, {gain, -}), %[keep] = {1 - fast, 1 - slow}, %[rates] = {fast, slow} (s); DC: %[dc] (+v), %[alpha],")
    print("// %[om2] = {1 - alpha, 1 - alpha}, %[a02] = {a0, a0} (s).  Clobbers v0-v53 (SDRG_CHUNK_CLOBBERS) and, for the")
    print("// AGC, vcc.")
    print("#pragma once")
    emit("SDRG_LPF_CHUNK_ASM", chunk("lpf"))
    emit("SDRG_AGC_CHUNK_ASM", chunk("agc"))
    emit("SDRG_DC_CHUNK_ASM", chunk("dc"))
    print("// the DC and AGC chunks with each quad's LDS write and read issued right after it (the product:")
    print("// SDRG_DC_ASM=2, SDRG_AGC_ASM=2; the grouped forms above are options 1)")
    emit("SDRG_DC_CHUNK_IL_ASM", chunk("dc", il=True))
    emit("SDRG_AGC_CHUNK_IL_ASM", chunk("agc", il=True))
    print("// the low-pass wave's whole loop with a one-chunk lookahead (SDRG_LPF_LOOKAHEAD; see lpf_loop() in the generator)")
    emit("SDRG_LPF_LOOP_ASM", lpf_loop())
    print("// the same loop with the chunk's LDS reads and writes interleaved quad by quad (SDRG_LPF_INTERLEAVE)")
    emit("SDRG_LPF_LOOP_IL_ASM", lpf_loop_interleaved())
    print("#define SDRG_CHUNK_CLOBBERS \\")
    regs = [f'"v{i}"' for i in range(T0 + 2)]
    for i in range(0, len(regs), 16):
        print("    " + ", ".join(regs[i:i + 16]) + (", \\" if i + 16 < len(regs) else ""))
    print("#define SDRG_LPF_CHUNK_CLOBBERS SDRG_CHUNK_CLOBBERS")
    print(f"#define SDRG_LPF_LOOP_SLOT_BYTES {SLOT}")


def main_lab():
    """tools/lab/lab_lpf_asm.h: lab-only forms of the low-pass chunk and loop (tools/lab/lpf_loop_lab.hip,
    tools/microbench/valu6.hip), included beside the product header; not in the product library"""
    print("// Generated by tools/gen/gen_lpf_asm.py --lab -- do not edit.  Lab only (tools/lab, tools/microbench; not in the")
    print("// product library): forms of the low-pass wave measured against the product's (DESIGN.md 3.3).  Include after")
    print("// csrc/ssb_lpf_asm.h (operands and clobbers as there).")
    print("#pragma once")
    print("// the interleaved loop on all 64 lanes, lane l running stream l mod 16 (four copies)")
    emit("SDRG_LPF_LOOP_IL_COPIES_ASM", lpf_loop_interleaved(copies=True))
    print("// the interleaved loop's VALU on all 64 lanes, its LDS operations on the 16 stream lanes")
    emit("SDRG_LPF_LOOP_IL_SPLIT_ASM", lpf_loop_interleaved(split=True))
    print("// the low-pass chunk with its VALU on all 64 lanes and the LDS operations on the caller's lanes; extra operand")
    print("// %[sv] (=&s, 64-bit): the caller's EXEC")
    emit("SDRG_LPF_CHUNK_SPLIT_ASM", chunk("lpf", split=True))
    print("// the low-pass chunk on register data, no LDS operations (wrong results), on the caller's lanes / on all 64 lanes")
    emit("SDRG_LPF_CHUNK_NOLDS_ASM", chunk("lpf", lds=False))
    emit("SDRG_LPF_CHUNK_NOLDS_SPLIT_ASM", chunk("lpf", lds=False, split=True))


if __name__ == "__main__":
    import sys
    main_lab() if "--lab" in sys.argv[1:] else main()
