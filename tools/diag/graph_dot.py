"""Diagnostic: the topology of a captured HIP graph (``DLBB_GRAPH_DOT=<path>`` makes
``FlatParamTrainer.capture_step`` dump it with ``hipGraphDebugDotPrint``). Reports kernel nodes,
forks / joins, the longest dependency chain in kernel nodes, and how many kernel nodes lie off
that chain (= could run beside it). One JSON line.

Usage: ``python tools/diag/graph_dot.py graph.dot``"""
import collections
import json
import re
import sys


def main(path):
    text = open(path).read()
    label = {}
    for m in re.finditer(r'"?([\w.]+)"?\s*\[([^\]]*)\]', text):
        nid, attrs = m.group(1), m.group(2)
        lab = re.search(r'label\s*=\s*"((?:[^"\\]|\\.)*)"', attrs)
        label[nid] = lab.group(1) if lab else ""
    edges = [(a, b) for a, b in re.findall(r'"?([\w.]+)"?\s*->\s*"?([\w.]+)"?', text)]
    succ, pred = collections.defaultdict(list), collections.defaultdict(list)
    nodes = set(label)
    for a, b in edges:
        succ[a].append(b)
        pred[b].append(a)
        nodes.update((a, b))

    def is_kernel(n):
        lab = label.get(n, "")
        return "KERNEL" in lab.upper() or "kernel" in lab

    order, indeg = [], {n: len(pred[n]) for n in nodes}
    q = collections.deque(n for n in nodes if indeg[n] == 0)
    while q:
        n = q.popleft()
        order.append(n)
        for s in succ[n]:
            indeg[s] -= 1
            if indeg[s] == 0:
                q.append(s)
    depth = {}
    for n in order:
        w = 1 if is_kernel(n) else 0
        depth[n] = w + max((depth[p] for p in pred[n]), default=0)
    kernels = [n for n in nodes if is_kernel(n)]
    longest = max(depth.values()) if depth else 0
    out = {"nodes": len(nodes), "edges": len(edges), "kernel_nodes": len(kernels),
           "forks": sum(1 for n in nodes if len(succ[n]) > 1),
           "joins": sum(1 for n in nodes if len(pred[n]) > 1),
           "longest_chain_kernels": longest,
           "kernels_off_longest_chain": len(kernels) - longest,
           "label_sample": [label[n][:80] for n in kernels[:3]]}
    print(json.dumps(out))


if __name__ == "__main__":
    main(sys.argv[1])
