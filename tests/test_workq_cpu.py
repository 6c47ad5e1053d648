"""Protocol model of the attention kernels' causal work queue (WorkQ in csrc/attention.hip),
run on the CPU: queue split, static first jobs, ticket fetches in random interleavings and the
reset-after-last-fetch rule. Every (block, head) job must run exactly once and every ticket must
be back at 0 after the launch, for any grid / head / block count (also fewer heads or
workgroups than queues)."""
import random

import pytest


def _launch(nwg, nblk, HB, xcd, tickets, rng):
    nq = 8 if xcd and HB >= 8 and nwg >= 8 else 1
    wgs = []
    for L in range(nwg):
        x = L % nq
        nwg_x = nwg // nq + (1 if x < nwg % nq else 0)
        hs = x * HB // nq
        hx = (x + 1) * HB // nq - hs
        njobs = hx * nblk
        wgs.append({"x": x, "hs": hs, "hx": hx, "njobs": njobs,
                    "base": min(nwg_x, njobs), "job": L // nq, "got": None})
    done = []
    live = [w for w in wgs if w["job"] < w["njobs"]]
    while live:
        w = rng.choice(live)
        if w["got"] is None:                      # job start: fetch the next ticket
            w["got"] = tickets[w["x"]]
            tickets[w["x"]] += 1
            jb, head = w["job"] // w["hx"], w["hs"] + w["job"] % w["hx"]
            done.append((jb, head))
        else:                                     # job end: publish, reset after the last fetch
            got, w["got"] = w["got"], None
            if got == w["njobs"] - 1:
                tickets[w["x"]] = 0
            w["job"] = w["base"] + got
            if w["job"] >= w["njobs"]:
                live.remove(w)
    return done


@pytest.mark.parametrize("nwg,nblk,HB", [(768, 8, 192), (6, 1, 6), (8, 8, 1), (64, 8, 8),
                                         (100, 16, 13), (7, 3, 20), (768, 32, 64), (1, 5, 3),
                                         (50, 2, 200)])
@pytest.mark.parametrize("xcd", [0, 1])
def test_every_job_once_and_tickets_reset(nwg, nblk, HB, xcd):
    rng = random.Random(nwg * 31 + nblk * 7 + HB + xcd)
    tickets = [0] * 8
    for _ in range(3):                            # back-to-back launches reuse the tickets
        nwg_eff = min(nwg, nblk * HB)             # the host's grid: min(jobs, resident cap)
        done = _launch(nwg_eff, nblk, HB, xcd, tickets, rng)
        assert sorted(done) == sorted((jb, h) for jb in range(nblk) for h in range(HB))
        assert tickets == [0] * 8


def test_heaviest_first_per_queue():
    """The static first jobs (workgroup rank r of a queue runs job r) are the heaviest blocks
    (jb 0 = heaviest) of the queue's heads: at the GPT-2 shape, blocks 0-3 of 8."""
    nwg, nblk, HB = 768, 8, 192
    for x in range(8):
        hx = (x + 1) * HB // 8 - x * HB // 8
        ranks = nwg // 8
        assert max(r // hx for r in range(ranks)) == 3
