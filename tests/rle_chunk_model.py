"""Numpy model of the encoder's lane-parallel MNP-5 pre-pass (hc_fgk.hip: rle_chunk).

Each 256-byte chunk is processed as 64 lanes x 4 bytes with a small carry between chunks; the
result must equal the serial FSM of transform.cpp:241-279 exactly. The model mirrors the kernel
step by step so that tests can check the algorithm on many random inputs on the CPU.

Per byte i of the chunk (c = diffed byte):
  same_i   = c_i == c_{i-1}        (i = 0: carry run counter R > 0 and c_0 == carried byte)
  start    = last i' <= i with !same_i'; with no start yet in the chunk the run began at
             -R_carry (k_0 = R_carry when the run continues)
  k_i      = i - start;  km = k_i mod 258
  R_i      = 0 if km == 257 (the 258-byte cut) else km + 1        (run counter after byte i)
  emitted  = final byte:  [R_{i-1} - 3 if R_{i-1} >= 3] + [c_i]
             km == 0:     [R_{i-1} - 3 if R_{i-1} >= 3] + [c_i]   (a run starts)
             km in {1,2}: [c_i]
             km == 257:   [255]
             else:        []
"""
import numpy as np


def rle_chunked(data, diff=False, chunk=256, fast=False):
    data = np.frombuffer(bytes(data), dtype=np.uint8).astype(np.int64)
    n = data.size
    out = []
    prev_x, R_carry, c_carry = 0, 0, 0
    for base in range(0, n, chunk):
        x = data[base:base + chunk]
        m = x.size
        xp = np.concatenate([[prev_x], x[:-1]])
        c = (x - xp) & 255 if diff else x.copy()
        fin = (base + m == n)
        if fast and m == chunk and not fin and (c == c_carry).all():
            sym, R_carry = pure_chunk(R_carry, c_carry)
            out += list(sym)
            prev_x = int(x[-1])
            continue
        cp = np.concatenate([[c_carry], c[:-1]])
        same = (c == cp)
        same[0] = R_carry > 0 and c[0] == c_carry
        idx = np.arange(m)
        starts = np.where(~same, idx, -1 << 30)
        last_start = np.maximum.accumulate(np.maximum(starts, -R_carry))
        k = idx - last_start
        km = np.where(k >= 258, k - 258, k)
        assert (k < 516).all()
        R = np.where(km == 257, 0, km + 1)
        Rprev = np.concatenate([[R_carry], R[:-1]])
        fin = (base + m == n)
        for i in range(m):
            final = fin and i == m - 1
            if final or km[i] == 0:
                if Rprev[i] >= 3:
                    out.append(int(Rprev[i] - 3))
                out.append(int(c[i]))
            elif km[i] in (1, 2):
                out.append(int(c[i]))
            elif km[i] == 257:
                out.append(255)
        prev_x, R_carry, c_carry = int(x[-1]), int(R[-1]), int(c[-1])
    return bytes(out)


def pure_chunk(R, c):
    """The encoder's fast path (hc_fgk.hip rle_chunk) for a full, non-final chunk whose 256 diffed
    bytes all equal the carried byte c: byte i sits at km = (R + i) mod 258, so the chunk emits
    only the events of the residues 257 (the cut: 255), 0, 1, 2 (c) that fall on i <= 255, in
    byte order: the cyclic order 257, 0, 1, 2 rotated to start at R when R <= 2 (lane j of the
    kernel takes entry j). Returns (symbols, run counter after the chunk)."""
    rot = R + 1 if R <= 2 else 0
    out = []
    for j in range(4):
        q = (j + rot) & 3
        e = 257 if q == 0 else q - 1
        i = e + 258 - R
        i = i - 258 if i >= 258 else i
        if i <= 255:
            out.append(255 if e == 257 else c)
    return bytes(out), (R + 256) % 258


# ---- 2 KB blocks for run-heavy streams (hc_fgk.hip: rle_block, HC_SPARSE_KB) --------------
#
# A full, non-final block (kBlock bytes: 2 KB as the kernel, 1 KB its other build) with few run starts (<= kSparseStarts) is coded by segments instead
# of byte by byte. Its bytes split at the run starts p_0 < .. < p_{S-1}: the carried segment
# [0, p_0) continues the run before the block (byte i at k = R + i, R the carried run counter) and
# segment j = [p_j, p_{j+1}) is a new run (k = i - p_j). Per byte, with km = k mod 258:
#   a run start emits [count R' - 3 if R' >= 3] + c   (R' = the run counter before it)
#   otherwise km in {0, 1, 2} emits c, km == 257 emits 255, the rest nothing
# so a segment emits, in order, its start's [count] + events at the offsets whose residue is in
# {0, 1, 2, 257}: the t-th of those (after the count) is 255 when t % 4 == 3, else c (a new run:
# residues 0, 1, 2, 257, 258 = 0, ...); the carried segment's start at residue R instead. The run
# counter before start j is (R + p_0) mod 258 for j = 0 and L_{j-1} mod 258 after a new run of
# length L_{j-1}. The kernel gives each start a lane and each event a lane (<= 63 events).
kBlock = 2048
kSparseStarts = 16


def n_events(L):
    """events of a new run's first L bytes (offsets with residue 0, 1, 2 or 257 mod 258)"""
    return 4 * (L // 258) + min(L % 258, 3)


def carried_events(R, L):
    """the carried segment: symbols of its first L bytes (byte i at residue (R + i) mod 258), c
    standing for the run byte (0x100) and 255 for a cut, in byte order (lane t of the kernel:
    cycle t >> 2, entry t & 3 of the cyclic order 257, 0, 1, 2 rotated to start at R)"""
    rot = R + 1 if R <= 2 else 0
    out = []
    for t in range(16 * kBlock // 1024):  # (the kernel's lanes t < 16 kQ)
        q = (t + rot) & 3
        e = 257 if q == 0 else q - 1
        i = (e - R) % 258 + 258 * (t >> 2)
        if i < L:
            out.append(255 if e == 257 else 0x100)
    return out


def sparse_block(c, c_carry, R):
    """c: the block's kBlock diffed bytes. Returns (symbols, R after the block), or None when the
    block has more than kSparseStarts starts or more than 63 symbols (the kernel then codes it as
    256-byte chunks)."""
    c = np.asarray(c, dtype=np.int64)
    prev = np.concatenate([[c_carry], c[:-1]])
    start = c != prev
    start[0] = start[0] or R == 0
    p = np.flatnonzero(start)
    S = p.size
    if S > kSparseStarts:
        return None
    L0 = int(p[0]) if S else kBlock
    syms = [c_carry if s == 0x100 else s for s in carried_events(R, L0)]
    ends = list(p[1:]) + [kBlock]
    for j in range(S):
        L = int(ends[j] - p[j])
        Rp = (R + int(p[0])) % 258 if j == 0 else int(p[j] - p[j - 1]) % 258
        if Rp >= 3:
            syms.append(Rp - 3)
        syms += [255 if t % 4 == 3 else int(c[p[j]]) for t in range(n_events(L))]
    if len(syms) > 63:
        return None
    Rn = (R + kBlock) % 258 if S == 0 else (kBlock - int(p[-1])) % 258
    return bytes(syms), Rn


def rle_blocked(data, diff=False, blocks=None):
    """The kernel's chunk loop for a stream that fits one buffer window: 256-byte chunks
    (rle_chunked's per-chunk rule) until a chunk has at most kSparseEnter starting lanes, then
    blocks of kBlock bytes while they are sparse and a whole block of full chunks remains before
    the last one; a dense block goes back to 256-byte chunks. `blocks`, when a list, receives
    (byte offset, carried run counter R) of every block coded sparse."""
    kb = kBlock // 256
    data = np.frombuffer(bytes(data), dtype=np.uint8).astype(np.int64)
    n = data.size
    nch = (n + 255) // 256
    out = []
    prev_x, R_carry, c_carry = 0, 0, 0
    ci, sparse = 0, False

    def diffed(x, px):
        xp = np.concatenate([[px], x[:-1]])
        return (x - xp) & 255 if diff else x.copy()

    while ci < nch:
        if sparse and ci + kb < nch:
            x = data[256 * ci:256 * ci + kBlock]
            c = diffed(x, prev_x)
            r = sparse_block(c, c_carry, R_carry)
            if r is not None:
                if blocks is not None:
                    blocks.append((256 * ci, R_carry))
                sym, R_carry = r
                out += list(sym)
                prev_x, c_carry = int(x[-1]), int(c[-1])
                ci += kb
                continue
            sparse = False
        base = 256 * ci
        x = data[base:base + 256]
        m = x.size
        # one chunk of rle_chunked's loop, inline (same carry)
        xp = np.concatenate([[prev_x], x[:-1]])
        c = (x - xp) & 255 if diff else x.copy()
        fin = base + m == n
        cp = np.concatenate([[c_carry], c[:-1]])
        same = c == cp
        same[0] = R_carry > 0 and c[0] == c_carry
        idx = np.arange(m)
        starts = np.where(~same, idx, -1 << 30)
        last_start = np.maximum.accumulate(np.maximum(starts, -R_carry))
        k = idx - last_start
        km = np.where(k >= 258, k - 258, k)
        Rv = np.where(km == 257, 0, km + 1)
        Rprev = np.concatenate([[R_carry], Rv[:-1]])
        for i in range(m):
            if (fin and i == m - 1) or km[i] == 0:
                if Rprev[i] >= 3:
                    out.append(int(Rprev[i] - 3))
                out.append(int(c[i]))
            elif km[i] in (1, 2):
                out.append(int(c[i]))
            elif km[i] == 257:
                out.append(255)
        # lanes (4 bytes each) holding a run start
        lanes = len(set(int(i) >> 2 for i in np.flatnonzero(~same)))
        sparse = lanes <= kSparseEnter
        prev_x, R_carry, c_carry = int(x[-1]), int(Rv[-1]), int(c[-1])
        ci += 1
    return bytes(out)


kSparseEnter = 2  # a 256-byte chunk whose run starts sit in at most this many lanes
