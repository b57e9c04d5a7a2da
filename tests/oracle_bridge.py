"""Convert oracle decisions into the product's per-contig result records (test helper)."""
import numpy as np

from oracle import orgscorer_oracle as orc
from waafle_amd.engine import Results
from waafle_amd.lib import CALL_LGT, CALL_NO_LGT, CALL_UNCLASSIFIED


def _members(tails, lca):
    return [t[-1] if t else lca for t in tails]


def oracle_results(contigs, batch, tax):
    """contigs: {name: oracle ContigModel} -> Results aligned with `batch`."""
    nsys = len(batch.systems)
    res = Results.empty(batch.n_contigs, batch.n_hits, batch.n_loci, nsys)
    res.clade1[:] = -1
    res.clade2[:] = -1
    res.annot_hit[:] = -1
    row_to_hit = {int(r): i for i, r in enumerate(batch.hit_row.tolist())}
    for c, name in enumerate(batch.contig_names):
        C = contigs[name]
        l0 = int(batch.loc_off[c])
        assert len(C.loci) == int(batch.loc_off[c + 1]) - l0
        mbase = 2 * int(batch.hit_off[c]) + 2 * c
        one, two = C.best_one, C.best_two
        res.pair_evals[c] = C.pair_evals
        res.ppot_sum[c] = C.ppot_sum
        res.iterations[c] = C.iterations
        if one is not None and one.ok:
            res.call[c] = CALL_NO_LGT
            res.crit[c], res.rank[c] = one.crit, one.rank
            res.clade1[c] = tax.index[one.clade1]
            res.synteny[l0:l0 + len(C.loci)] = np.frombuffer(one.synteny.encode(), np.uint8)
            mem = _members(one.tails1, one.clade1)
            res.n_meld1[c] = len(mem)
            res.meld[mbase:mbase + len(mem)] = [tax.index[m] for m in mem]
        elif two is not None and two.ok:
            res.call[c] = CALL_LGT
            res.crit[c], res.rank[c] = two.crit, two.rank
            res.clade1[c] = tax.index[two.clade1]
            res.clade2[c] = tax.index[two.clade2]
            res.direction[c] = 1 if two.direction == "B>A" else 0
            res.synteny[l0:l0 + len(C.loci)] = np.frombuffer(two.synteny.encode(), np.uint8)
            m1 = sorted(set(_members(two.tails1, two.clade1)))
            m2 = sorted(set(_members(two.tails2, two.clade2)))
            res.n_meld1[c], res.n_meld2[c] = len(m1), len(m2)
            res.meld[mbase:mbase + len(m1)] = [tax.index[m] for m in m1]
            res.meld[mbase + len(m1):mbase + len(m1) + len(m2)] = [tax.index[m] for m in m2]
        else:
            res.call[c] = CALL_UNCLASSIFIED
        for g, L in enumerate(C.loci):
            for b, system in enumerate(batch.systems):
                row = L.annotation_rows.get(system)
                if row is not None:
                    res.annot_hit[(l0 + g) * nsys + b] = row_to_hit[row]
    return res


def run_oracle(paths, flags):
    from waafle_amd import cli
    params = orc.Params(**cli.param_dict(cli.parse_flags(flags)))
    return orc.run(*paths, params)


class _Hit:
    pass


def oracle_hits_from_batch(b, tax):
    """In-memory oracle hits for a packed batch (scores are already exact floats)."""
    groups = []
    for c, name in enumerate(b.contig_names):
        hs = []
        for i in range(int(b.hit_off[c]), int(b.hit_off[c + 1])):
            h = _Hit()
            h.qstart, h.qend = int(b.hit_qlo[i]), int(b.hit_qhi[i])
            h.strand = "-" if b.hit_strand[i] else "+"
            h.scov_mod = float(b.hit_scov[i])
            h.score = float(b.hit_score[i])
            h.taxon = tax.names[int(b.hit_taxon[i])]
            vid = int(b.annot_value_ids[i, 0])
            h.annotations = {"UniProt": b.annot_values[0][vid]} if vid >= 0 else {}
            h.order = int(b.hit_row[i])
            hs.append(h)
        if hs:
            groups.append((name, hs))
    return groups


def oracle_loci_from_batch(b):
    groups = []
    for c, name in enumerate(b.contig_names):
        ls = []
        for l in range(int(b.loc_off[c]), int(b.loc_off[c + 1])):
            st = {0: "+", 1: "-"}.get(int(b.loc_strand[l]), ".")
            ls.append(orc.GeneLocus([name, "x", "gene", str(int(b.loc_start[l])),
                                     str(int(b.loc_end[l])), ".", st, "0", "."]))
        if ls:
            groups.append((name, ls))
    return groups
