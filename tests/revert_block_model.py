"""Model of the decoder's lane-parallel RLE + diff revert (hc_fgk.hip: revert_block).

The serial revert of transform.cpp:137-159 (then the diff revert of transform.cpp:231-239) is a
4-state machine on r = run counter: a symbol read in state 3 is a count (it emits `count`
copies of the previous symbol, r -> 0); otherwise it is a literal, r -> r + 1 when it equals
the previous symbol and r is 1 or 2, else r -> 1. Each symbol's transition is one of two
functions on {0,1,2,3}, stored as a 4-byte table (byte x = f(x)), so g o f is one byte
permute of g by f (v_perm_b32); functions compose, so a wave-wide inclusive scan of the
compositions gives every symbol's state. Output lengths (1 or count) and diff sums (symbol, or
count x previous symbol, mod 256) are plain scans. Bytes are emitted in two passes: every
literal writes its byte; a lane holds at most one count (a count follows three equal literals,
so counts are >= 4 symbols apart), whose run -- an arithmetic sequence mod 256 with the diff
model, a constant without -- the whole wave writes 64 bytes at a time.

`revert_blocked(symbols, diff)` mirrors the kernel: blocks of 256 symbols, 64 lanes x 4, a carry
of (state, last symbol, last output byte) between blocks.
"""

F_EQ = 1 | 2 << 8 | 3 << 16 | 0 << 24   # r: 0->1, 1->2, 2->3, 3->0 (count)
F_NE = 1 | 1 << 8 | 1 << 16 | 0 << 24   # r: 0->1, 1->1, 2->1, 3->0
F_ID = 0 | 1 << 8 | 2 << 16 | 3 << 24   # past the block's end


def perm(s1, sel):
    """v_perm_b32(0, s1, sel) for selector bytes 0..3: byte i = byte sel[i] of s1"""
    return sum(((s1 >> (8 * ((sel >> (8 * i)) & 255))) & 255) << (8 * i) for i in range(4))


def compose(g, f):
    """x -> g(f(x))"""
    return perm(g, f)


def apply(f, r):
    return (f >> (8 * r)) & 255


def revert_blocked(symbols, diff):
    sym = list(symbols)
    out = bytearray()
    r_c, last_c, prev_c = 0, 0, 0
    for base in range(0, len(sym), 256):
        blk = sym[base:base + 256]
        m = len(blk)
        blk = blk + [0] * (256 - m)
        prevsym = [last_c] + blk[:-1]
        f = [(F_EQ if blk[i] == prevsym[i] else F_NE) if i < m else F_ID for i in range(256)]
        # per lane: F = f3 o f2 o f1 o f0
        lanes = []
        for l in range(64):
            F = F_ID
            for b in range(4):
                F = compose(f[4 * l + b], F)
            lanes.append(F)
        # inclusive scan (Hillis-Steele, as the kernel does it with shuffles)
        inc = lanes[:]
        off = 1
        while off < 64:
            inc = [compose(inc[l], inc[l - off]) if l >= off else inc[l] for l in range(64)]
            off *= 2
        exc = [F_ID] + inc[:-1]
        # state before each symbol, output lengths and diff sums
        r_before = [0] * 256
        for l in range(64):
            r = apply(exc[l], r_c)
            for b in range(4):
                i = 4 * l + b
                r_before[i] = r
                r = apply(f[i], r)
        count = [i < m and r_before[i] == 3 for i in range(256)]
        length = [(blk[i] if count[i] else 1) if i < m else 0 for i in range(256)]
        dsum = [((blk[i] * prevsym[i]) if count[i] else blk[i]) & 255 if i < m else 0 for i in range(256)]
        lane_len = [sum(length[4 * l:4 * l + 4]) for l in range(64)]
        lane_d = [sum(dsum[4 * l:4 * l + 4]) & 255 for l in range(64)]
        start = [sum(lane_len[:l]) for l in range(64)]
        dstart = [(prev_c + sum(lane_d[:l])) & 255 for l in range(64)]
        blk_out = bytearray(sum(lane_len))
        runs = []
        for l in range(64):
            p, prev = start[l], dstart[l]
            assert sum(count[4 * l:4 * l + 4]) <= 1
            for b in range(4):
                i = 4 * l + b
                if count[i]:  # the run: its offset, length, first value and step
                    c, n_ = prevsym[i], length[i]
                    if n_:
                        runs.append((p, n_, prev if diff else c, c if diff else 0))
                    prev = (prev + n_ * c) & 255 if diff else (c if n_ else prev)
                    p += n_
                elif i < m:  # a literal
                    prev = ((prev if diff else 0) + blk[i]) & 255
                    blk_out[p] = prev
                    p += 1
        for p, n_, base, step in runs:  # the wave, 64 bytes at a time
            for j0 in range(0, n_, 64):
                for j in range(j0, min(n_, j0 + 64)):
                    blk_out[p + j] = (base + step * (j + 1)) & 255
        out += blk_out
        r_c = apply(inc[63], r_c)
        last_c = blk[m - 1]
        prev_c = (prev_c + sum(lane_d)) & 255 if diff else (blk_out[-1] if blk_out else prev_c)
    return bytes(out)
