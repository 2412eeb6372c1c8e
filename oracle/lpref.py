"""Plain-Python restatement of the reference's link-prediction sample loops
(evaluation_util.py:84-158) driving a ``random.Random`` instance call for
call as the reference drives the module-level one. TEST INFRASTRUCTURE ONLY:
the checker of libhgx's hgx_pyrandom_* (which must leave the generator in
the same state and pick the same pairs)."""


def sample_missing_connections(hypergraph, num_samples, rnd):
  """evaluation_util.py:125-158 (random.choice twice per try, set of
  accepted pairs, 10 x num_samples tries)."""
  n_nodes, n_edges = len(hypergraph.node), len(hypergraph.edge)
  assert num_samples < n_nodes * n_edges
  assert n_edges > 0 and n_nodes > 0
  node_list = list(hypergraph.node)
  edge_list = list(hypergraph.edge)
  members = {n: set(hypergraph.node[n].edges) for n in node_list}
  picked = set()
  budget = 10 * num_samples
  while budget and len(picked) < num_samples:
    budget -= 1
    n = rnd.choice(node_list)
    e = rnd.choice(edge_list)
    if e in members[n]:
      continue
    picked.add((n, e))
  return list(picked)


def remove_random_connections(hypergraph, probability, rnd):
  """evaluation_util.py:84-122 on plain dicts: returns (node -> remaining
  edge list, edge -> remaining node list, removed pairs in order)."""
  node_edges = {n: list(v.edges) for n, v in hypergraph.node.items()}
  edge_nodes = {e: list(v.nodes) for e, v in hypergraph.edge.items()}
  candidates = [(n, e) for n in node_edges for e in node_edges[n]]
  rnd.shuffle(candidates)
  removed = []
  for n, e in candidates:
    if len(node_edges[n]) == 1 or len(edge_nodes.get(e, [])) == 1:
      continue
    if rnd.random() < probability and probability > 0:
      node_edges[n].remove(e)
      edge_nodes[e].remove(n)
      removed.append((n, e))
  return node_edges, edge_nodes, removed
