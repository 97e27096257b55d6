"""CPU checks of the one-process multi-GPU multiply's event graph (csrc/multi.hip run_ranks).

mpfft_multi_schedule replays `calls` back-to-back mpfft_mul_multi_device calls as a dry run
(no GPU touched) and returns every event record, stream wait, queued kernel and peer copy.
These tests rebuild the happens-before graph of HIP streams and events from it (stream order
plus record -> wait edges, a wait binding the event's most recent record) and check:
  - every copy pulls from a rank only after that rank produced what is pulled;
  - phase 1 of the combine (the stripe carries) waits for phase 0 of every rank and never
    for another rank's phase 1 (the ranks' phase 1 were chained);
  - nothing of call k+1 on rank e runs before call k's pulls from rank e on the other ranks'
    streams are done (a write-after-read race between back-to-back calls);
and that both properties fail on mutants of the graph that reintroduce the old orderings.
"""
import pytest

SHAPES = [(17, 2, 156250000, 156250000),   # C4
          (13, 32, 1000000, 999000), (15, 4, 2000000, 1900000), (10, 1, 2000, 1800)]

# what a copy pulls from rank e, and the work on e that produces it
PRODUCER = {"xchg1": "fwd_columns_a", "xchg2": "inv_rows", "halo": "halo_pack", "sums": "combine0"}


def graph(tr):
    """nodes (call, kind, rank, stream, what, src) and each node's ancestor set (int bitset)"""
    nodes, anc = [], []
    last = {}       # stream -> last node
    rec = {}        # (rank, event) -> node of its latest record
    call = 0
    for t in tr:
        if t[0] == "N":
            call += 1
            continue
        kind, d, st = t[0], t[1], t[2]
        i = len(nodes)
        a = 0
        p = last.get((d, st))
        if p is not None:
            a |= anc[p] | (1 << p)
        if kind == "W":
            r = rec.get((t[3], t[4]))
            if r is not None:
                a |= anc[r] | (1 << r)
        what = t[3] if kind in "KC" else t[-1]
        src = t[4] if kind == "C" else (t[3] if kind == "W" else d)
        nodes.append((call, kind, d, st, what, src))
        anc.append(a)
        last[(d, st)] = i
        if kind == "R":
            rec[(d, t[3])] = i
    return nodes, anc


def before(anc, a, b):
    return bool((anc[b] >> a) & 1)


def violations(tr, world):
    nodes, anc = graph(tr)
    bad = []
    idx = lambda **k: [i for i, n in enumerate(nodes)
                       if all(n[("call", "kind", "rank", "stream", "what", "src").index(f)] == v for f, v in k.items())]
    calls = max(n[0] for n in nodes) + 1
    for c in range(calls):
        # a pull from e follows e's producer
        for i in idx(call=c, kind="C"):
            _, _, d, _, what, e = nodes[i]
            if e == d or what not in PRODUCER:
                continue
            prod = idx(call=c, kind="K", rank=e, what=PRODUCER[what])
            if not prod or not all(before(anc, j, i) for j in prod):
                bad.append(("pull before producer", c, d, what, e))
        # phase 1 after every phase 0, and unchained from the others' phase 1
        p0 = {d: idx(call=c, kind="K", rank=d, what="combine0")[0] for d in range(world)}
        p1 = {d: idx(call=c, kind="K", rank=d, what="combine1")[0] for d in range(world)}
        for d in range(world):
            for e in range(world):
                if not before(anc, p0[e], p1[d]):
                    bad.append(("phase 1 before a phase 0", c, d, e))
                if e != d and before(anc, p1[e], p1[d]):
                    bad.append(("phase 1 chained", c, d, e))
        # exchange #1's pulls from e done before e's inverse columns overwrite e's column arrays
        for i in idx(call=c, kind="C", what="xchg1"):
            e = nodes[i][5]
            for j in idx(call=c, kind="K", rank=e, what="inv_columns"):
                if not before(anc, i, j):
                    bad.append(("column arrays overwritten before exchange #1 pulled them", c, e))
        # call c's pulls from e done before anything of call c + 1 on e
        if c + 1 < calls:
            for i in idx(call=c, kind="C"):
                _, _, d, _, what, e = nodes[i]
                if e == d:
                    continue
                for j, n in enumerate(nodes):
                    if n[0] == c + 1 and n[2] == e and n[1] in "KC" and not before(anc, i, j):
                        bad.append(("next call overtakes a pull", c, d, what, e, n[4]))
                        break
    return bad


@pytest.mark.parametrize("world", [2, 4, 8])
@pytest.mark.parametrize("depth,w,n1,n2", SHAPES)
def test_event_graph(mp, world, depth, w, n1, n2):
    tr = mp.multi_schedule(n1, n2, depth, w, world, calls=3)
    kinds = {t[0] for t in tr}
    assert kinds == {"R", "W", "K", "C", "N"}
    assert not violations(tr, world)


@pytest.mark.parametrize("world", [2, 8])
def test_event_graph_mutants_fail(mp, world):
    depth, w, n1, n2 = SHAPES[0]
    tr = mp.multi_schedule(n1, n2, depth, w, world, calls=2)
    # round 5's phase 1: the summary pulls waited on `ev`, which each rank re-records after its
    # own phase 1 inside the same loop
    chained = [t[:4] + ("ev",) if t[0] == "W" and t[4] == "evs" else t for t in tr]
    chained = [t[:3] + ("ev",) if t[0] == "R" and t[3] == "evs" else t for t in chained]
    assert any(v[0] == "phase 1 chained" for v in violations(chained, world))
    # round 5's call start: no wait on the other ranks' end of the previous call
    racy = [t for t in tr if not (t[0] == "W" and t[4] == "evd")]
    assert any(v[0] == "next call overtakes a pull" for v in violations(racy, world))


def test_schedule_rejects_bad_worlds(mp):
    with pytest.raises(mp.MpfftError):
        mp.multi_schedule(2000, 1800, 10, 1, 3)
