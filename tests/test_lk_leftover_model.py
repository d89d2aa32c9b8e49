"""CPU model of the background LK grid's leftover list (track.hip
lk_item_kernel: give_back / the drain's close).  Resident waves hand items
whose frame is not ready to a list; the end-of-chunk drain runs them.  Every
atomic step of the device protocol is one step of a Python generator, and a
scheduler interleaves the waves (random seeds plus the adversarial schedule
ADVICE r04 describes: a give-back after the drain has read the count).

The model of the current protocol (count reserved by CAS on an open count,
the drain closes the count with atomicOr, a resident wave that finds the list
closed runs its item itself) must run every item exactly once under every
schedule; the model of the round-4 protocol (atomicAdd reservation, the drain
reads the count once) is shown to lose an item under the adversarial one.
"""
from __future__ import annotations

import random

CLOSED = 1 << 30


class Mem:
    def __init__(self):
        self.count = 0       # bg_left[1]
        self.cursor = 0      # bg_left[0]
        self.slots = {}      # bg_left[32 + j] -> item
        self.ran = []


def resident_new(m: Mem, items):
    """A resident wave whose frame wait timed out: give back its items (the
    dequeued one and the pending second), or run them when the list is
    closed (every ready flag is up once the drain runs)."""
    for it in items:
        c = m.count
        yield
        while True:
            if c & CLOSED:
                m.ran.append(it)  # run_item(..., must)
                yield
                break
            # atomicCAS(count, c, c + 1)
            prev = m.count
            if prev == c:
                m.count = c + 1
                yield
                m.slots[c] = it  # publish (relaxed store)
                yield
                break
            c = prev
            yield


def drain_new(m: Mem, closer: bool = True):
    """The drain's first wave closes the list (atomicOr) and publishes the
    count it read in one word (bg_left[2]); every other drain wave waits for
    that word."""
    if closer:
        n = m.count & ~CLOSED
        m.count |= CLOSED  # atomicOr, returns the count before
        yield
        m.published = n
        yield
    else:
        while getattr(m, "published", None) is None:
            yield
        n = m.published
        yield
    while True:
        j = m.cursor
        m.cursor += 1
        yield
        if j >= n:
            return
        while j not in m.slots:  # bounded wait on the publication
            yield
        m.ran.append(m.slots[j])
        yield


def resident_old(m: Mem, items):
    for it in items:
        j = m.count
        m.count += 1  # atomicAdd reservation
        yield
        m.slots[j] = it
        yield


def drain_old(m: Mem):
    n = m.count  # read once
    yield
    while True:
        j = m.cursor
        m.cursor += 1
        yield
        if j >= n:
            return
        while j not in m.slots:
            yield
        m.ran.append(m.slots[j])
        yield


def run(waves, order=None, seed=0, max_steps=100000):
    """Step the generators to completion; `order` (wave indices) first, then
    random choices.  A waiting drain wave keeps yielding, so every schedule
    terminates once the producers are done."""
    rng = random.Random(seed)
    live = list(range(len(waves)))
    order = list(order or [])
    steps = 0
    while live and steps < max_steps:
        steps += 1
        w = order.pop(0) if order else rng.choice(live)
        if w not in live:
            continue
        try:
            next(waves[w])
        except StopIteration:
            live.remove(w)
    return not live


def test_leftover_list_runs_every_item_once_under_random_schedules():
    for seed in range(400):
        m = Mem()
        items = [[("r0", 0), ("r0", 1)], [("r1", 0), ("r1", 1)], [("r2", 0)]]
        rng = random.Random(seed)
        # some resident give-backs happen before the drain, some race it
        early = [resident_new(m, it) for it in items[:1]]
        for g in early:
            while True:
                try:
                    next(g)
                except StopIteration:
                    break
        waves = [resident_new(m, it) for it in items[1:]] + [drain_new(m, closer=(d == 0))
                                                            for d in range(rng.randint(1, 3))]
        assert run(waves, seed=seed), f"seed {seed}: a wave never finished"
        want = sorted(x for it in items for x in it)
        assert sorted(m.ran) == want, f"seed {seed}: ran {sorted(m.ran)}"


def test_give_back_after_the_drain_read_the_count():
    # adversarial order: drain 2 (index 1) closes and reads the count first,
    # then the resident wave (index 0) gives back, then drain 2 steps
    m = Mem()
    waves = [resident_new(m, [("r", 0)]), drain_new(m)]
    assert run(waves, order=[1, 0, 0, 0, 0, 1, 1, 1, 1])
    assert m.ran == [("r", 0)]


def test_round4_protocol_loses_that_item():
    m = Mem()
    waves = [resident_old(m, [("r", 0)]), drain_old(m)]
    assert run(waves, order=[1, 0, 0, 1, 1, 1])
    assert m.ran == []  # the item landed past the count the drain read


def decode(head, k, n, n_frames):
    """track.hip lk_item_kernel's item numbers of head `head`: (frame, point)
    or None (padding / the last frame's dummy numbers)."""
    seg = (n + 7) // 8
    base = (n_frames - 1) * seg
    base_e = base + (base & 1)
    if k < base:
        f = k // seg
        i = head * seg + (k - f * seg)
    else:
        r = k - base_e
        if r < 0 or r & 1:
            return None
        f, i = n_frames - 1, head * seg + r // 2
    return (f, i) if i < n else None


def test_head_numbers_cover_every_item_once_and_split_the_last_frame():
    for n in (1, 7, 8, 9, 2465, 5325):
        for n_frames in (1, 2, 3, 20, 64):
            seg = (n + 7) // 8
            base = (n_frames - 1) * seg
            per_head = base + (base & 1) + 2 * seg
            seen = []
            for head in range(8):
                for k0 in range(0, per_head, 2):  # two-number dequeues from 0
                    got = [decode(head, k, n, n_frames) for k in (k0, k0 + 1) if k < per_head]
                    got = [g for g in got if g is not None]
                    seen += got
                    # no dequeue carries two points of the last frame
                    assert sum(1 for f, _ in got if f == n_frames - 1) <= 1
            assert sorted(seen) == [(f, i) for f in range(n_frames) for i in range(n)]
