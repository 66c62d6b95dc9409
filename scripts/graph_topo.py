import re, sys, collections
s = open(sys.argv[1]).read()
nodes = {}
for m in re.finditer(r'"(graph_\d+_node_\d+)"\[style="\w+"shape="record"label="\{\n(\w+)\n\| \{ID \| \d+ \| ([^\\|}]*)', s):
    name = m.group(3).strip()
    dm = re.search(r'(\w+?kernel\w*?)E', name)
    short = re.sub(r'_ZN3tdp12_GLOBAL__N_1\d+', '', name)[:40]
    nodes[m.group(1)] = (m.group(2), short)
for m in re.finditer(r'"(graph_\d+_node_\d+)"\[style="\w+"shape="record"label="\{\n(\w+)\n', s):
    if m.group(1) not in nodes: nodes[m.group(1)] = (m.group(2), "")
edges = re.findall(r'"(graph_\d+_node_\d+)" -> "(graph_\d+_node_\d+)"', s)
succ = collections.defaultdict(list); pred = collections.defaultdict(list)
for a, b in edges: succ[a].append(b); pred[b].append(a)
# topo order
indeg = {n: len(pred[n]) for n in nodes}
q = [n for n in nodes if indeg[n] == 0]; order = []
while q:
    n = q.pop(0); order.append(n)
    for b in succ[n]:
        indeg[b] -= 1
        if indeg[b] == 0: q.append(b)
idx = {n: i for i, n in enumerate(order)}
lim = int(sys.argv[2]) if len(sys.argv) > 2 else 10**9
for n in order[:lim]:
    k, nm = nodes[n]
    print(f"{idx[n]:3d} {k[:6]:6s} {nm:40s} <- {[idx[p] for p in pred[n]]} -> {[idx[x] for x in succ[n]]}")
print(len(nodes), "nodes", len(edges), "edges")
