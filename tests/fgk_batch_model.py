"""Model of the FGK kernels' batched hot paths (hc_fgk.hip: the encoder's code_all_batch, the
decoder's Dec::decode_batch), checked against the reference's update (huffman.cpp:95-128, which
the slot-form Tree.update equals: tests/test_cache_model.py).

Between swaps and splits the tree's shape is fixed, and the update of a symbol whose every level
passes the lane-parallel leader test only adds 1 to the weights on its root path. Such updates
commute, so a batch of symbols is tested at once. Exactly (batch_len): symbol j's test at position
a uses the weights before the batch plus one per earlier batch symbol whose path holds a (c0) or
a + 1 (c1). The kernels test conservatively (tentative_len): every batch symbol's increments are
added first, so a position's word counts all batch symbols through it (c0 at its largest), and the
next position's word is the one read before (c1 = 0): a level can be reported falsely, never passed
when it fails. The first symbol with a reported level (or no cached path / no leaf in the tables)
ends the batch; the symbols before it commit (+1 on every path position, the root once each) and it
is coded alone, exactly as the one-symbol loop codes it.

retry_len (HC_BATCH_RETRY) adds the kernels' retest: when the first failing symbol jf > 0 may have
failed falsely -- an earlier batch symbol holds the next position a + 1 of its first failing level
(the test counted c1 = 0), or a later one holds a (counted as earlier) -- the symbols before it are
committed and the tentative test runs again on symbols jf.., now with their exact counts at every
position, for as long as it moves jf on. grad -c -m (four symbols, ties on every row): 1034 batches
and 523 symbols alone per stream -> 671 and 15.
"""
from fgk_cache_model import ROOT, PathCache, Tree, _word

BATCH = 7  # the encoder: seven cached symbols per step (groups of nine lanes)


def batch_len(t, paths):
    """paths: root paths (ROOT last) of up to BATCH cached symbols, None for an uncached one;
    the kernel's jf: the first symbol that fails, len(paths) if none"""
    for j, p in enumerate(paths):
        if p is None:
            return j
        for a in p:
            if a == ROOT:
                break
            c0 = sum(1 for q in paths[:j] if a in q)
            c1 = sum(1 for q in paths[:j] if a + 1 != ROOT and (a + 1) in q)
            if not _word(t, a + 1) + 1024 * c1 >= _word(t, a) + 1024 * c0 + 1024:
                return j
    return len(paths)


def retry_len(t, paths):
    """the kernels' tentative test with the retest (module docstring): jf, never past batch_len"""
    jmax = len(paths)
    for j, p in enumerate(paths):
        if p is None:
            jmax = j
            break
    j0 = 0
    while True:
        com, cnt = {}, {}
        for q in paths[:j0]:  # committed: exact
            for a in q:
                com[a] = com.get(a, 0) + 1
        for q in paths[j0:jmax]:  # tentative
            for a in q:
                cnt[a] = cnt.get(a, 0) + 1

        def word(a):
            return _word(t, a) + 1024 * com.get(a, 0)
        jf, fa = jmax, None
        for j in range(j0, jmax):
            for a in paths[j]:
                if a != ROOT and word(a + 1) < word(a) + 1024 * cnt[a]:
                    jf, fa = j, a
                    break
            if fa is not None:
                break
        if jf >= jmax or jf == j0:
            return jf
        if not (any((fa + 1) in q for q in paths[:jf]) or any(fa in q for q in paths[jf + 1:jmax])):
            return jf
        j0 = jf


SMALL_NYT = ROOT - 32  # small-alphabet batches while at most 16 symbols are seen (positions >= 480)
SMALL_G, SMALL_K = 4, 15  # ... with four lanes per symbol (depth <= 4) and fifteen symbols per step


def small_len(t, paths):
    """the encoder's small-alphabet batch (hc_fgk.hip code_small): exact counts -- symbol j's test
    at position a counts the earlier batch symbols through a (c0) and through a + 1 (c1; every
    earlier one when a + 1 is the root) from membership marks -- so jf = the first symbol whose
    update would swap (or end at the NYT's parent), exactly as the one-symbol loop finds it"""
    for j, p in enumerate(paths):
        if p is None:
            return j
        for a in p:
            if a == ROOT:
                break
            c0 = sum(1 for q in paths[:j] if a in q)
            c1 = j if a + 1 == ROOT else sum(1 for q in paths[:j] if (a + 1) in q)
            if t.w[a + 1] + c1 < t.w[a] + c0 + 1:
                return j
    return len(paths)


def encode(symbols, batched, misses=False, lanes=9, exact=False, retry=False, small=False):
    """(codes, tree, stats): every symbol's code bits and the final tree; batched=False is the
    one-symbol loop, True the batched one (the kernel's tentative test; exact=True: exact counts).
    misses=True (measured and dropped): a symbol that has a leaf but no cached path joins the batch
    with its chased root path (if it fits `lanes` levels with the root) and is inserted into the
    path cache once committed."""
    t = Tree()
    pc = PathCache()
    codes = []
    stats = {"batches": 0, "alone": 0}

    def code_path(pv, fresh, sym):
        code = [p & 1 for p in reversed(pv)]
        return code[:-1] + [(sym >> k) & 1 for k in range(7, -1, -1)] if fresh else code

    def alone(sym):
        fresh = t.where[sym] == 0
        if fresh:
            t.split(sym)
        x = t.where[sym]
        pv = pc.lookup(sym)
        if pv is None:
            pv = t.path(x)
            pc.insert(sym, pv)
        codes.append(code_path(pv, fresh, sym))
        t.update(x)
        for s, lead in t.swaps:
            pc.on_swap(s, lead)

    def cached(sym, depth=99):
        e = pc.slot.get(sym)
        if t.where[sym] == 0:
            return None
        if e is None:
            if not misses:
                return None
            p = t.path(t.where[sym]) + [ROOT]
            return p if len(p) <= lanes else None
        return pc.ent[e][1] + [ROOT] if len(pc.ent[e][1]) <= depth else None

    i, n = 0, len(symbols)
    while i < n:
        if not batched:
            alone(symbols[i])
            i += 1
            continue
        if small and t.nyt >= SMALL_NYT:  # exact batches of up to SMALL_K symbols of depth <= SMALL_G
            paths = []
            for s_ in symbols[i:i + SMALL_K]:
                paths.append(cached(s_, SMALL_G))
                if paths[-1] is None:
                    break
            jf = small_len(t, paths)  # (more exact than batch_len, which never counts the root as c1)
            stats["small"] = stats.get("small", 0) + 1
            for p in paths[:jf]:
                codes.append([a & 1 for a in reversed(p[:-1])])
                for a in p:
                    t.w[a] += 1
            i += jf
            if jf < len(paths):
                stats["alone"] += 1
                alone(symbols[i])
                i += 1
            continue
        paths = [cached(s) for s in symbols[i:i + BATCH]]
        jf = batch_len(t, paths) if exact else (retry_len if retry else tentative_len)(t, paths)
        assert jf <= batch_len(t, paths)
        stats["batches"] += 1
        for s_, p in zip(symbols[i:i + jf], paths[:jf]):
            codes.append([a & 1 for a in reversed(p[:-1])])
            for a in p:
                t.w[a] += 1
            if misses and pc.slot.get(s_) is None:
                pc.insert(s_, p[:-1])
        i += jf
        if jf < len(paths):
            stats["alone"] += 1
            alone(symbols[i])
            i += 1
    return codes, t, stats


# ---- the decoder's batched hot path (hc_fgk.hip: Dec::decode_batch)

DEC_BATCH = 6
TABLE_DEPTH = 8  # the level tables reach codes of up to 8 bits


def tentative_len(t, paths):
    """paths: root paths (ROOT last) of a batch's symbols, None for one without a cached path (the
    encoder) or whose table entry is no leaf (the decoder); the kernels' jf. Every batch symbol's
    increment is added tentatively, so a position's word after the adds counts all batch symbols
    through it (c0 at its largest, every one of them counted as earlier) while the next position's
    word is the one read before (c1 = 0): a level fails when word(a + 1) < word(a) + 1024 * C(a)."""
    cnt = {}
    for p in paths:
        if p is None:
            break
        for a in p:
            cnt[a] = cnt.get(a, 0) + 1
    for j, p in enumerate(paths):
        if p is None:
            return j
        for a in p:
            if a != ROOT and _word(t, a + 1) < _word(t, a) + 1024 * cnt[a]:
                return j
    return len(paths)


def decode(symbols, batched, retry=False):
    """(tree, stats): decode the stream of `symbols` (the model knows them; the kernel reads them
    from the tables) with the one-symbol loop or with batches, returning the final tree. Batch
    symbols are those whose code is at most TABLE_DEPTH bits and leads to a leaf."""
    t = Tree()
    stats = {"batches": 0, "alone": 0}

    def alone(sym):
        if t.where[sym] == 0:
            t.split(sym)
        t.update(t.where[sym])

    i, n = 0, len(symbols)
    while i < n:
        if not batched:
            alone(symbols[i])
            i += 1
            continue
        paths = []
        for s in symbols[i:i + DEC_BATCH]:
            x = t.where[s]
            p = t.path(x) if x else None
            if p is None or len(p) > TABLE_DEPTH:
                paths.append(None)
                break
            paths.append(p + [ROOT])
        jf = (retry_len if retry else tentative_len)(t, paths)
        assert jf <= batch_len(t, paths + [None])  # never passes what the exact test fails
        stats["batches"] += 1
        for p in paths[:jf]:
            for a in p:
                t.w[a] += 1
        i += jf
        if jf < len(paths):
            stats["alone"] += 1
            alone(symbols[i])
            i += 1
    return t, stats
