"""GPU: the warm device-sized build and its hipGraph replay.

A warm build runs the digest and the whole tail on the counts the digest left
on the device (one host sync, after the last kernel); the second identical
warm build of a bounded digest is captured as a hipGraph and every later one
replays it.  Every build of these sequences must equal the oracle: plain,
capture, replays, a different proteome in between (new key: plain again), a
bigger one (the reservation grows: the build is redone), timing of one stage
(event nodes in the graph) and the graph switched off (option build_graph=0);
with depth bins (the default for warm tryptic builds) and the radix tail."""
from __future__ import annotations

import numpy as np
import pytest

from dbindex_amd import fasta
from dbindex_amd.params import DBIndexSearchParams
from oracle import cref
from tests.helpers import assert_index_equal, assert_queries_equal, query_masses

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def env():
    from dbindex_amd import _native
    from dbindex_amd._native import DeviceBuffer, synchronize
    from dbindex_amd.engine import Engine
    if _native.device_count() == 0:
        pytest.fail("no HIP device visible: the gpu tests need an MI355X")
    return Engine, DeviceBuffer, synchronize


def _dev(env, pp):
    _, DeviceBuffer, synchronize = env
    d_res = DeviceBuffer.from_numpy(np.concatenate([pp.residues, np.zeros(16, np.uint8)]), 0)
    d_off = DeviceBuffer.from_numpy(pp.offsets.astype(np.uint64), 0)
    synchronize(0)
    return d_res, d_off


@pytest.mark.parametrize("graph,depth", [(1, 1), (0, 1), (1, 0)])
def test_warm_builds_and_graph_replays_match_oracle(env, graph, depth):
    Engine = env[0]
    hum = fasta.config("human")
    a, b = hum.slice(0, 6000), hum.slice(6000, 9000)
    big = hum.slice(0, 14000)
    cp = DBIndexSearchParams.trypsin(2).to_c()
    oa, ob, obig = (cref.Index(cp, p.residues, p.offsets) for p in (a, b, big))
    bufs = {id(p): _dev(env, p) for p in (a, b, big)}

    def build(eng, p):
        d_res, d_off = bufs[id(p)]
        return eng.build_device(d_res.ptr, p.n_residues, d_off.ptr, p.n_proteins)

    with Engine(cp, options={"build_graph": graph, "depth_bins": depth}) as eng:
        eng.set_timing(False)
        seq = [a, a, a, a, a, b, b, b, a, a, big, big, big, a]
        want = {id(a): oa, id(b): ob, id(big): obig}
        for k, p in enumerate(seq):
            st = build(eng, p)
            assert st.n_total == want[id(p)].n_total, k
            assert_index_equal(eng, want[id(p)], f"graph={graph} depth={depth} build {k}")
        m, t = query_masses(oa, 3000, seed=21)
        assert_queries_equal(eng, oa, m, t, f"graph={graph} queries after replays")
        # one stage timed: event nodes inside the graph
        eng.set_timing(True, only="digest")
        for k in range(4):
            build(eng, a)
            assert_index_equal(eng, oa, f"graph={graph} timed build {k}")
            times = {name: ms for name, ms, _ in eng.stage_times()}
            assert times.get("digest", 0.0) > 0.0 and times.get("radix_scatter", 0.0) == 0.0


@pytest.mark.parametrize("graph,depth", [(1, 1), (0, 1), (1, 0)])
def test_replays_over_rewritten_inputs(env, graph, depth):
    """A caller that rewrites its residues IN PLACE (a reused staging buffer:
    same d_res, n_res, n_prot) replays the captured graph over new contents.
    Nothing the graph bakes in depends on the contents -- grids and buffers
    are sized from capacities, every kernel reads the real counts on the
    device -- and whatever the new contents outgrow (digest slots, chunk-list
    grids, a first giant chunk) is caught by the one host check and the build
    is redone.  Every build must equal the oracle of what the buffer holds."""
    Engine, _, synchronize = env
    a = fasta.config("human").slice(0, 6000)
    # B: the same offsets over the residues reversed (other peptides, other counts)
    b = fasta.PackedProteins(a.residues[::-1].copy(), a.offsets.copy(), a.defs)
    # C: the first 250 proteins rewritten as GAAAAAAK repeats -- equal-mass
    # spikes of ~11 k records each: giant chunks the earlier builds never had
    spike = a.residues.copy()
    e250 = int(a.offsets[250])
    pat = np.frombuffer(b"GAAAAAAK", np.uint8)
    spike[:e250] = np.resize(pat, e250)
    c = fasta.PackedProteins(spike, a.offsets.copy(), a.defs)
    cp = DBIndexSearchParams.trypsin(2).to_c()
    want = {k: cref.Index(cp, p.residues, p.offsets) for k, p in (("a", a), ("b", b), ("c", c))}
    assert want["c"].n_total > want["a"].n_total
    d_res, d_off = _dev(env, a)
    contents = {"a": a, "b": b, "c": c}
    with Engine(cp, options={"build_graph": graph, "depth_bins": depth}) as eng:
        eng.set_timing(False)
        seq = ["a", "a", "a", "a", "b", "b", "b", "c", "c", "c", "c", "a", "a", "b", "c"]
        cur = "a"
        for k, name in enumerate(seq):
            if name != cur:  # rewrite the same device buffer
                d_res.upload(contents[name].residues)
                synchronize(0)
                cur = name
            st = eng.build_device(d_res.ptr, a.n_residues, d_off.ptr, a.n_proteins)
            assert st.n_total == want[name].n_total, (k, name)
            assert_index_equal(eng, want[name], f"graph={graph} depth={depth} build {k} ({name})")
        m, t = query_masses(want["c"], 2000, seed=5)
        assert_queries_equal(eng, want["c"], m, t, f"graph={graph} queries over the spiked proteome")
