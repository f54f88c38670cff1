#!/usr/bin/env python3
"""Model check of the party-parallel kernel's share ring (mkacc_quad.hpp, quadp_step).

One gate, k parties on G = ceil(k / ppw) workgroups (workgroup w owns parties
w ppw .. w ppw + ppw - 1), steps rel = 0 .. k n - 2 of one launch; the index party of
step rel is (rel + 1) // n (run_args: index = t / n with t = rel + 1) and the index
workgroup the one owning it.  Per step a workgroup runs its parties' passes, then:

  * not the index: waits for used >= rel + 1 - SLOTS, writes its tagged share of rel
    to slot rel % SLOTS, goes on to rel + 1;
  * the index: after its passes (or, with preload, also when its pass starts); on
    taking over from another party, first waits for used >= rel + 1 - SLOTS (and with
    preload loads again); takes the shares of rel, accepting a slot only when
    its tag equals 1 + rel mod 8 (zeroed slots never match) and reloading the others;
    in the last SLOTS steps of its turn writes its own share to its slot; posts used =
    rel + 1; goes on to rel + 1.

Random schedules (one enabled action at a time) must finish every step, never accept
a share of another step (a tag alias), and keep `used` monotonic.  The same model
with the index's own slot writes, the takeover wait or the reload after it removed
finds the stale-share failures that the first GPU runs of the tagged ring hit.

    python tools/quadp_protocol.py      # all checks; exit status 0 when clean
"""
from __future__ import annotations

import random
import sys

SLOTS, TAGS = 4, 8


def run(k: int, n: int, seed: int, own_write: bool = True, takeover_wait: bool = True,
        reload: bool = True, ppw: int = 1, preload: bool = False) -> str | None:
    rnd = random.Random(seed)
    steps = k * n - 1
    slot = {}                                 # (slot, workgroup) -> step written
    used = 0
    groups = -(-k // ppw)
    rel = [0] * groups
    phase = ["pass"] * groups
    seen: list[list] = [[] for _ in range(groups)]   # the index workgroup's loaded slots

    def load(w: int, r: int) -> list:
        return [slot.get((r % SLOTS, u)) for u in range(groups) if u != w]

    def index(r: int) -> int:
        return ((r + 1) // n) // ppw

    while True:
        if all(r >= steps for r in rel):
            return None
        moved = False
        for w in rnd.sample(range(groups), groups):
            r = rel[w]
            if r >= steps:
                continue
            if phase[w] == "pass":
                if w == index(r) and preload:
                    seen[w] = load(w, r)
                phase[w] = "after"
                moved = True
                break
            if w != index(r):
                if r + 1 > SLOTS and used < r + 1 - SLOTS:
                    continue
                slot[(r % SLOTS, w)] = r
            else:
                takeover = r > 0 and index(r - 1) != w
                if phase[w] == "after":
                    if takeover_wait and takeover and r + 1 > SLOTS and used < r + 1 - SLOTS:
                        continue
                    if (takeover and reload) or not preload:
                        seen[w] = load(w, r)
                    phase[w] = "take"
                got = seen[w]
                if not all(g is not None and g % TAGS == r % TAGS for g in got):
                    seen[w] = load(w, r)
                    moved = True
                    break
                if any(g != r for g in got):
                    return f"k={k} n={n} seed={seed}: step {r} took shares of steps {got}"
                if used > r + 1:
                    return f"k={k} n={n} seed={seed}: used went back from {used} to {r + 1}"
                if own_write and index(r + SLOTS) != w:
                    slot[(r % SLOTS, w)] = r
                used = r + 1
            rel[w] += 1
            phase[w] = "pass"
            moved = True
            break
        if not moved:
            return f"k={k} n={n} seed={seed}: deadlock at steps {rel}, used {used}"


def check(seeds: int = 200, ppws=(1,), **kw) -> list[str]:
    bad = []
    for k in (2, 3, 4, 5, 8, 16):
        for n in (1, 2, 3, 4, 5, 8, 9, 17, 40):
            for ppw in ppws:
                if k * n < 2 or -(-k // ppw) < 2:
                    continue
                for seed in range(seeds):
                    err = run(k, n, seed, ppw=ppw, **kw)
                    if err:
                        bad.append(err)
                        break
    return bad


def main() -> int:
    bad = check(ppws=(1, 2, 3, 4)) + check(seeds=60, ppws=(1, 2), preload=True)
    print(f"quadp share ring: {'clean' if not bad else bad[:3]}")
    weak = [check(seeds=60, own_write=False), check(seeds=60, takeover_wait=False),
            check(seeds=60, reload=False, preload=True)]
    print("failing shapes without the index's own slot writes / the takeover wait / (preloading) the reload:",
          [len(w) for w in weak])
    return 0 if not bad and all(weak) else 1


if __name__ == "__main__":
    sys.exit(main())
