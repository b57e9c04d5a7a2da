"""Interned taxonomy tables for the device (restates waafle/utils.py:374-447).

Every name that can appear as a clade (taxonomy file names, hit taxa, "r__Root",
"Unknown") gets an id equal to its rank in Python code-point order, so the
reference's `clade1 < clade2` string comparison (orgscorer.py:608) and its sorted
output are integer comparisons on the device.
"""
import csv

import numpy as np

ROOT = "r__Root"        # utils.py:368
UNKNOWN = "Unknown"     # utils.py:367


class TaxonomyError(ValueError):
    pass


def read_edges(path):
    """2-column TSV, csv excel-tab dialect (utils.py:379-382)."""
    edges = []
    with open(path) as fh:
        for row in csv.reader(fh, csv.excel_tab):
            if len(row) != 2:   # upstream's tuple unpacking raises here
                raise TaxonomyError("taxonomy row must have 2 columns: {}".format(row))
            edges.append((row[0], row[1]))
    return edges


class TaxonomyTables:
    """parent/depth/sibling-parent/leaf-count arrays over interned ids."""

    def __init__(self, edges, extra_names=()):
        parents = {}
        children = {}
        listed_under = {}
        for child, parent in edges:
            parents[child] = parent                          # last line wins (:381)
            children.setdefault(parent, set()).add(child)    # every line counts (:382)
            listed_under.setdefault(child, set()).add(parent)
        names = set(parents) | set(children) | {ROOT, UNKNOWN} | set(extra_names)
        self.names = sorted(names)
        self.index = {n: i for i, n in enumerate(self.names)}
        n = len(self.names)
        idx = self.index
        self.root = idx[ROOT]
        self.unknown = idx[UNKNOWN]
        self._parents = parents
        self._children = children
        self.parent = np.array([idx[parents.get(nm, ROOT)] for nm in self.names], dtype=np.int32)

        # depth = len(get_lineage) - 1: walk parents until r__Root (:392-399)
        depth = np.full(n, -1, dtype=np.int64)
        depth[self.root] = 0
        par = self.parent
        for i in range(n):
            if depth[i] >= 0:
                continue
            path = []
            x = i
            seen = set()
            while depth[x] < 0:
                if x in seen:
                    raise TaxonomyError(
                        "taxonomy cycle through {!r}: lineage never reaches {}".format(
                            self.names[x], ROOT))
                seen.add(x)
                path.append(x)
                x = int(par[x])
            d = depth[x]
            for y in reversed(path):
                d += 1
                depth[y] = d
        self.depth = depth.astype(np.int32)

        # sisters = children(parent(x)) - {x} (:428-434): a clade s is a sister of x iff
        # s is listed under parent(x).  A clade listed under two parents is rejected.
        sib = np.full(n, -1, dtype=np.int32)
        for child, under in listed_under.items():
            if len(under) > 1:
                raise TaxonomyError("clade {!r} listed under several parents: {}".format(
                    child, sorted(under)))
            sib[idx[child]] = idx[next(iter(under))]
        self.sib_parent = sib

        # leaf counts (:436-447): 1 when a clade has no listed children
        leaf = np.zeros(n, dtype=np.int64)
        state = np.zeros(n, dtype=np.int8)    # 0 new, 1 open, 2 done
        kids = {idx[p]: [idx[c] for c in cs] for p, cs in children.items()}
        for start in range(n):
            if state[start]:
                continue
            stack = [(start, False)]
            while stack:
                x, expanded = stack.pop()
                if state[x] == 2:
                    continue
                ks = kids.get(x)
                if ks is None:
                    leaf[x] = 1
                    state[x] = 2
                elif expanded:
                    leaf[x] = sum(int(leaf[k]) for k in ks)
                    state[x] = 2
                else:
                    if state[x] == 1:
                        raise TaxonomyError("taxonomy children cycle through {!r}".format(
                            self.names[x]))
                    state[x] = 1
                    stack.append((x, True))
                    for k in ks:
                        if state[k] == 1:
                            raise TaxonomyError("taxonomy children cycle through {!r}".format(
                                self.names[k]))
                        if state[k] == 0:
                            stack.append((k, False))
        self.leaf_count = leaf
        self._lineage_cache = {}

    # ---- host-side string helpers for rendering ---------------------------------
    def lineage(self, i):
        """Names from r__Root down to id i (utils.py:392-399)."""
        got = self._lineage_cache.get(i)
        if got is None:
            path = [i]
            while path[-1] != self.root:
                path.append(int(self.parent[path[-1]]))
            got = [self.names[x] for x in reversed(path)]
            self._lineage_cache[i] = got
        return got

    def lca(self, ids):
        paths = [self.lineage(i) for i in ids]
        best = ROOT
        for level in zip(*paths):
            if len(set(level)) != 1:
                break
            best = level[0]
        return best

    def tail(self, i, lca_name):
        """get_tails for one clade (utils.py:413-426) as a list of names."""
        path = self.lineage(i)
        if lca_name in path:
            path = path[len(path) - path[::-1].index(lca_name):]
        return path
