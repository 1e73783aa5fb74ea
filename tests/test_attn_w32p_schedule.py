"""CPU model of the persistent prefill attention kernel's schedule (attention.hip,
attn_prefill_w32p_kernel, prefill version 9): the same item walk, LDS block-id lists and LDS-DMA
ring bookkeeping as the kernel, replayed in Python for random batches, checking what a mistake
would only show on the GPU as a fault or slightly-off rows:

* every (sequence, kv head, row tile) with rows is run exactly once, over all workgroups;
* a tile is staged only from a block-id list that holds its item's ids (the next item's list is
  written in the current item's prologue -- round 6 faulted when a one-tile item let the switch
  stage the item after next from a list not yet written);
* every tile is staged before its iteration waits for it, at most one tile is in flight behind it
  when the wait is vmcnt(4), and a ring slot is overwritten only after the barrier that follows the
  last read of its previous tile (K in its iteration, V^T in the next one or the item's tail).
"""
import random

NB = 4            # ring depth
KBS = 32          # keys per block


def items_of(wg, grid, ngroups, nx, hkv, cu, seq_lens, rwg):
    """The kernel's pos_of / load_item / next_item for workgroup wg: [(item fields), ...]."""
    xcd, wx, px = wg & 7, wg >> 3, grid >> 3
    gx = (ngroups - 1 - xcd) // 8 + 1 if ngroups > xcd else 0
    nitems = gx * nx
    out = []
    r = 0
    while True:
        p = r * px + ((px - 1 - wx) if r & 1 else wx)
        if p >= nitems:
            break
        gi, qt = p // nx, nx - 1 - p % nx
        g = xcd + 8 * gi
        b, kvh = g // hkv, g % hkv
        qs, ql = cu[b], cu[b + 1] - cu[b]
        row0 = qt * rwg
        if row0 < ql:
            qpos0 = seq_lens[b] - ql
            kmax = qpos0 + min(row0 + rwg, ql) - 1
            nch = kmax // KBS + 1
            out.append(dict(b=b, kvh=kvh, qt=qt, ntile=(nch + 1) // 2))
        r += 1
    return out


def replay(items):
    """The kernel's staging control flow over one workgroup's items; returns the event log."""
    ev = []                                # (kind, ...) in program order (uniform control flow)
    lists = {0: None, 1: None}             # block-id list -> item index it holds
    staged_tiles = {}                      # global tile -> (item index, local tile, time)
    g0, staged, il = 0, 0, 0
    k = 0                                  # index of cur in items
    time = [0]

    def stage_global(gidx, may_next, cur_k):
        nonlocal staged
        lt = gidx - g0
        cur = items[cur_k]
        if lt < cur["ntile"]:
            it, lst, t = cur_k, il, lt
        elif may_next and cur_k + 1 < len(items) and lt - cur["ntile"] < items[cur_k + 1]["ntile"]:
            it, lst, t = cur_k + 1, il ^ 1, lt - cur["ntile"]
        else:
            return
        assert lists[lst] == it, f"tile {gidx} of item {it} staged from list {lst} holding {lists[lst]}"
        assert gidx not in staged_tiles and gidx == staged
        staged_tiles[gidx] = (it, t, time[0])
        staged = gidx + 1

    if not items:
        return staged_tiles
    lists[0] = 0
    time[0] = -1                                   # before the first barrier
    stage_global(0, False, 0)
    stage_global(1, False, 0)
    while True:
        cur = items[k]
        if k + 1 < len(items):
            lists[il ^ 1] = k + 1                  # prologue: the next item's list
        for t in range(cur["ntile"]):
            gidx = g0 + t
            assert staged > gidx, f"tile {gidx} not staged at its wait"
            if staged > gidx + 1:
                assert staged <= gidx + 2          # vmcnt(4): exactly one tile behind it
            time[0] = 2 * gidx + 1                 # after iteration gidx's barrier
            if staged == gidx + 1:
                stage_global(gidx + 1, True, k)
            if staged == gidx + 2:
                stage_global(gidx + 2, True, k)
        if k + 1 >= len(items):
            break
        g0 += cur["ntile"]
        k += 1
        il ^= 1
        time[0] = 2 * (g0 - 1) + 1.5               # the switch: after the last iteration's code
        while staged < g0 + 2:
            before = staged
            stage_global(staged, False, k)
            if staged == before:
                break
    total = sum(it["ntile"] for it in items)
    assert sorted(staged_tiles) == list(range(total))
    for x, (_, _, tm) in staged_tiles.items():
        if x >= NB:
            # slot of tile x - NB: K read in iteration x - NB, V^T in x - NB + 1 (or the tail, before
            # the next prologue's __syncthreads, i.e. before iteration x - NB + 1's barrier); every wave
            # is past those reads after iteration x - NB + 2's barrier
            assert tm >= 2 * (x - NB + 2) + 1, (x, tm)
    return staged_tiles


def _batch(rng):
    b = rng.randint(1, 12)
    hkv = rng.choice([1, 2, 8])
    ql = [rng.choice([1, 5, 31, 64, 65, 128, 200, 700]) for _ in range(b)]
    ctx = [q + rng.choice([0, 0, 17, 300]) for q in ql]
    cu = [0]
    for q in ql:
        cu.append(cu[-1] + q)
    return b, hkv, ql, ctx, cu


def test_persistent_prefill_schedule_is_complete_and_safe():
    rng = random.Random(0)
    for _ in range(300):
        b, hkv, ql, ctx, cu = _batch(rng)
        g = rng.choice([1, 2, 4, 8, 16])
        rwg = 8 * (32 // g)
        nx = (max(ql) + rwg - 1) // rwg
        grid = rng.choice([8, 16, 64, 256])
        ngroups = b * hkv
        seen = []
        for wg in range(grid):
            its = items_of(wg, grid, ngroups, nx, hkv, cu, ctx, rwg)
            replay(its)
            seen += [(it["b"], it["kvh"], it["qt"]) for it in its]
        want = [(bb, h, qt) for bb in range(b) for h in range(hkv) for qt in range(nx) if qt * rwg < ql[bb]]
        assert sorted(seen) == sorted(want)


def test_one_tile_items_do_not_stage_past_the_written_lists():
    """The round-6 fault's shape: 128-token prompts at G = 4 alternate two-tile and one-tile items."""
    items = [dict(b=0, kvh=0, qt=q, ntile=n) for q, n in enumerate([2, 1, 2, 1, 1, 1, 2, 1])]
    staged = replay(items)
    assert len(staged) == 11
