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


def chunk(role, lds=True, split=False):
    """role 'dc', 'lpf' or 'agc'.  split (low-pass, lab): VALU with all 64 lanes on (lanes past the 16 streams compute on whatever their
    registers hold and store nothing), LDS operations with the caller's EXEC (saved in %[sv])"""
    out = []

    def exec_lds(ops):
        return ([f"s_mov_b64 exec, %[sv]"] + ops + ["s_mov_b64 exec, -1"]) if (split and ops) else ops

    if split:
        out += ["s_mov_b64 %[sv], exec"]
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
                continue
            if role == "lpf":
                out += lpf_sample(b + q, prev1, prev2)
                prev2, prev1 = prev1, pair(b + q)
            else:
                out += agc_sample(b + q, g)
                g = b + q
        if lds:
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
    print("// the low-pass chunk with its VALU on all 64 lanes and the LDS operations on the caller's lanes; extra operand")
    print("// %[sv] (=&s, 64-bit): the caller's EXEC (lab option SDRG_LPF_ASM=2)")
    emit("SDRG_LPF_CHUNK_SPLIT_ASM", chunk("lpf", split=True))
    print("// lab only (tools/microbench/valu6.hip): the low-pass chunk on register data, no LDS operations")
    emit("SDRG_LPF_CHUNK_NOLDS_ASM", chunk("lpf", lds=False))
    print("#define SDRG_CHUNK_CLOBBERS \\")
    regs = [f'"v{i}"' for i in range(T0 + 2)]
    for i in range(0, len(regs), 16):
        print("    " + ", ".join(regs[i:i + 16]) + (", \\" if i + 16 < len(regs) else ""))
    print("#define SDRG_LPF_CHUNK_CLOBBERS SDRG_CHUNK_CLOBBERS")


if __name__ == "__main__":
    main()
