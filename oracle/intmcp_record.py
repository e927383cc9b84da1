"""Per-step record of an I-NTMCP planner (shared by the reference harness, the
oracle and the GPU tests).  TEST INFRASTRUCTURE (see ``oracle/__init__.py``).

Hashes cover the level-1 root's particles (t, state words, the other agent's
history as (action | -1, obs key) steps) and, for each distinct other-agent
history in that belief (first-occurrence order), the level-0 node's visits,
registered children (registration order) and particles.  Nesting level 2 adds
``nested2``: the third tree's history of every particle of those second-tree
nodes, in order, and each distinct such node's visits, children and
particles; nesting level 3 adds ``nested3``, the same one tree further down."""
import hashlib
import json
import struct


def _fhex(x):
    return float(x).hex()


def hist_digest(h):
    m = hashlib.sha1()
    for a, k in h:
        m.update(struct.pack("<iQ", a, k))
    return m.hexdigest()


def _node_entry(h, node):
    if node is None:
        return [hist_digest(h), None]
    visits, nkids, nparts = node
    mm = hashlib.sha1()
    for t, (v0, v1) in nparts:
        mm.update(struct.pack("<III", t, v0, v1))
    return [hist_digest(h), int(visits), [[a, int(v), _fhex(val)] for a, v, val in nkids],
            len(nparts), mm.hexdigest()]


def intmcp_record(rec, num_sims, search_depth, root_visits, kids, mn, mx, parts, nested_nodes,
                  full=False, nested2=None, deeper=()):
    """nested2 (nesting level >= 2): (per second-tree node of nested_nodes, the
    third-tree histories of its particles in order; [(history, node)] of the
    distinct third-tree nodes, first-occurrence order).  deeper: the same for
    the fourth tree (from the third tree's nodes) and on, recorded as
    nested3_*, ..."""
    rec["num_sims"] = num_sims
    if num_sims > 0:
        rec["search_depth"] = search_depth
        rec["root_visits"] = int(root_visits)
        rec["children"] = [[a, int(v), _fhex(val), _fhex(tot)] for a, v, val, tot in kids]
        rec["min_value"] = _fhex(mn)
        rec["max_value"] = _fhex(mx)
    m = hashlib.sha1()
    for t, (v0, v1), h in parts:
        m.update(struct.pack("<III", t, v0, v1))
        m.update(hist_digest(h).encode())
    rec["belief_size"] = len(parts)
    rec["belief_digest"] = m.hexdigest()
    out = [_node_entry(h, node) for h, node in nested_nodes]
    rec["nested_count"] = len(out)
    rec["nested_digest"] = hashlib.sha1(json.dumps(out, separators=(",", ":")).encode()).hexdigest()
    if full:
        rec["nested"] = out
    if nested2 is not None:
        seqs, nodes2 = nested2
        o2 = [[[hist_digest(h) for h in seq] for seq in seqs],
              [_node_entry(h, node) for h, node in nodes2]]
        rec["nested2_count"] = len(nodes2)
        rec["nested2_digest"] = hashlib.sha1(json.dumps(o2, separators=(",", ":")).encode()).hexdigest()
    for d, (seqs, nodes) in enumerate(deeper, start=3):
        od = [[[hist_digest(h) for h in seq] for seq in seqs],
              [_node_entry(h, node) for h, node in nodes]]
        rec[f"nested{d}_count"] = len(nodes)
        rec[f"nested{d}_digest"] = hashlib.sha1(json.dumps(od, separators=(",", ":")).encode()).hexdigest()
    return rec
