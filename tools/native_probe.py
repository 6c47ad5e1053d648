import os, sys, time, torch
sys.path.insert(0, os.getcwd())
from distributed_llm_backend_benchmark_amd.parallel.comm import init_distributed
from distributed_llm_backend_benchmark_amd.parallel.collectives import make_op, make_data
comm = init_distributed("rccl")
x = make_data((1 << 29,), torch.bfloat16, 0, comm.device)
for name in ("sendrecv", "allgather"):
    op = make_op(name, comm, x, impl="native")
    out = op.recv if name == "sendrecv" else op.out
    out.zero_()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    s.record(); op.run(); e.record(); e.synchronize()
    t1 = time.perf_counter()
    ok = bool(torch.equal(out.view(-1)[:1000], x.view(-1)[:1000])) and bool(torch.equal(out.view(-1)[-1000:], x.view(-1)[-1000:]))
    print(name, "event us", s.elapsed_time(e) * 1e3, "host us", (t1 - t0) * 1e6, "copied", ok)
    torch.cuda.synchronize()
    t0 = time.perf_counter(); op.run(); torch.cuda.synchronize(); print(name, "host+sync us", (time.perf_counter() - t0) * 1e6)
comm.destroy()
