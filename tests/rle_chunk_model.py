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
