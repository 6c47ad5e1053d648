"""Diagnostic: does HIP-graph replay run the parallel branches of a captured
fork / join concurrently? Two independent chains of spin kernels (``torch.cuda._sleep``), one on
the current stream and one on a side stream forked / joined by events — the pattern of the
DDP step's side-stream weight gradients — timed eager and as one replayed graph. Concurrent
branches take ~one chain's time, serialised branches ~two. Also the same with two streams of
small GEMM chains (work that occupies only part of the GPU, like the wgrad kernels).

Prints one JSON line: eager / graph ms for both workloads, the ratio to one chain's time, and the
HIP graph env knobs in force (DEBUG_HIP_FORCE_GRAPH_QUEUES, DEBUG_CLR_GRAPH_PACKET_CAPTURE).
"""
import json
import os

import torch


def timed(fn, iters=10):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / iters


def main():
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    side = torch.cuda.Stream(dev)
    out = {"env": {k: os.environ.get(k) for k in ("DEBUG_HIP_FORCE_GRAPH_QUEUES",
                                                   "DEBUG_CLR_GRAPH_PACKET_CAPTURE",
                                                   "GPU_MAX_HW_QUEUES")}}
    a = torch.randn(2048, 2048, device=dev, dtype=torch.bfloat16)
    b = torch.randn(2048, 2048, device=dev, dtype=torch.bfloat16)
    c1 = torch.empty_like(a)
    c2 = torch.empty_like(a)
    cyc = 200_000
    work = {"sleep": (lambda: torch.cuda._sleep(cyc), lambda: torch.cuda._sleep(cyc)),
            "gemm": (lambda: torch.matmul(a, b, out=c1), lambda: torch.matmul(b, a, out=c2))}
    for name, (w1, w2) in work.items():
        n = 8
        one = timed(lambda: [w1() for _ in range(n)])

        def step():
            cur = torch.cuda.current_stream()
            side.wait_stream(cur)
            for _ in range(n):
                w1()
            with torch.cuda.stream(side):
                for _ in range(n):
                    w2()
            cur.wait_stream(side)
        eager = timed(step)
        cap = torch.cuda.Stream(dev)
        cap.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(cap):
            step()
        torch.cuda.current_stream().wait_stream(cap)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            step()
        graph = timed(g.replay)
        out[name] = {"one_chain_ms": round(one, 4), "eager_ms": round(eager, 4),
                     "graph_ms": round(graph, 4), "eager_over_one": round(eager / one, 3),
                     "graph_over_one": round(graph / one, 3)}
    # the DDP backward's pattern: every "layer" forks a side-stream kernel off the main chain
    # mid-graph (side.wait_stream(main) before each), one join at the end
    for name, (w1, w2) in work.items():
        L = 8

        def layers():
            cur = torch.cuda.current_stream()
            for _ in range(L):
                w1()
                side.wait_stream(cur)
                with torch.cuda.stream(side):
                    w2()
            cur.wait_stream(side)
        one = timed(lambda: [w1() for _ in range(L)])
        eager = timed(layers)
        cap = torch.cuda.Stream(dev)
        cap.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(cap):
            layers()
        torch.cuda.current_stream().wait_stream(cap)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            layers()
        graph = timed(g.replay)
        out[name + "_midgraph_forks"] = {"one_chain_ms": round(one, 4), "eager_ms": round(eager, 4),
                                         "graph_ms": round(graph, 4),
                                         "eager_over_one": round(eager / one, 3),
                                         "graph_over_one": round(graph / one, 3)}
    # how many forks can one graph hold before the replay stops overlapping its branches? (the
    # GPT-2 step forks the side stream ~50 times; the probes above fork 8 times)
    if os.environ.get("GB_FORK_SWEEP", "1") == "1":
        short = 20_000
        for L in (8, 16, 32, 64, 128):
            def many():
                cur = torch.cuda.current_stream()
                for _ in range(L):
                    torch.cuda._sleep(short)
                    side.wait_stream(cur)
                    with torch.cuda.stream(side):
                        torch.cuda._sleep(short)
                cur.wait_stream(side)
            one = timed(lambda: [torch.cuda._sleep(short) for _ in range(L)])
            eager = timed(many)
            cap = torch.cuda.Stream(dev)
            cap.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(cap):
                many()
            torch.cuda.current_stream().wait_stream(cap)
            torch.cuda.synchronize()
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                many()
            graph = timed(g.replay)
            out[f"sleep_forks_L{L}"] = {"one_chain_ms": round(one, 4), "eager_ms": round(eager, 4),
                                        "graph_ms": round(graph, 4),
                                        "eager_over_one": round(eager / one, 3),
                                        "graph_over_one": round(graph / one, 3)}
    # the same with the side kernels dealt round-robin over k side streams: a side node then
    # depends on the main chain and on the side node k layers back, not the one just before
    sides = [side] + [torch.cuda.Stream(dev) for _ in range(3)]
    for k in (2, 4):
        for name, (w1, w2) in work.items():
            L = 8

            def layers_rr():
                cur = torch.cuda.current_stream()
                for i in range(L):
                    w1()
                    sd = sides[i % k]
                    sd.wait_stream(cur)
                    with torch.cuda.stream(sd):
                        w2()
                for sd in sides[:k]:
                    cur.wait_stream(sd)
            one = timed(lambda: [w1() for _ in range(L)])
            eager = timed(layers_rr)
            cap = torch.cuda.Stream(dev)
            cap.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(cap):
                layers_rr()
            torch.cuda.current_stream().wait_stream(cap)
            torch.cuda.synchronize()
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                layers_rr()
            graph = timed(g.replay)
            out[f"{name}_midgraph_forks_rr{k}"] = {
                "one_chain_ms": round(one, 4), "eager_ms": round(eager, 4),
                "graph_ms": round(graph, 4), "eager_over_one": round(eager / one, 3),
                "graph_over_one": round(graph / one, 3)}
    # does one memcpy / memset node anywhere in the graph change how its branches run? (the
    # GPT-2 step's graph holds D2D copies and fills besides kernels)
    src_buf = torch.randn(1 << 20, device=dev)
    dst_buf = torch.empty_like(src_buf)
    for extra in ("memcpy", "memset"):
        def forks_extra():
            cur = torch.cuda.current_stream()
            if extra == "memcpy":
                dst_buf.copy_(src_buf)                 # hipMemcpyAsync D2D -> memcpy node
            else:
                torch.cuda.current_stream()            # noqa
                dst_buf.zero_()                        # fill (kernel or memset node)
            side.wait_stream(cur)
            for _ in range(8):
                torch.cuda._sleep(cyc)
            with torch.cuda.stream(side):
                for _ in range(8):
                    torch.cuda._sleep(cyc)
            cur.wait_stream(side)
        one = timed(lambda: [torch.cuda._sleep(cyc) for _ in range(8)])
        eager = timed(forks_extra)
        cap = torch.cuda.Stream(dev)
        cap.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(cap):
            forks_extra()
        torch.cuda.current_stream().wait_stream(cap)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            forks_extra()
        graph = timed(g.replay)
        out[f"sleep_forks_with_{extra}"] = {
            "one_chain_ms": round(one, 4), "eager_ms": round(eager, 4), "graph_ms": round(graph, 4),
            "eager_over_one": round(eager / one, 3), "graph_over_one": round(graph / one, 3)}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
