"""Native GraphML ingestion: shd_graphml_parse vs the
harness reader (shdpe.graph.read_graphml, igraph's import order) and the
committed fixtures.  Host-only: no GPU needed.

tests/data/topology.graphml.xml.xz is Shadow's shipped topology
(resource/topology.graphml.xml.xz, a data file), the input of
tests/golden/shipped_topology.npz."""
import os

import numpy as np
import pytest

from shdpe import generators as G
from shdpe.engine import EngineError, parse_graphml
from shdpe.graph import Topology, read_graphml, write_graphml

DATA = os.path.join(os.path.dirname(__file__), "data")
GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def same(a: Topology, b: Topology):
    assert a.n == b.n and a.m == b.m and a.directed == b.directed
    assert a.prefers_direct == b.prefers_direct
    assert np.array_equal(a.src, b.src) and np.array_equal(a.dst, b.dst)
    for x, y in ((a.latency, b.latency), (a.loss, b.loss)):
        assert np.array_equal(x.view(np.int64), y.view(np.int64))   # bit-exact, NaN included
    assert (a.vloss is None) == (b.vloss is None)
    if a.vloss is not None:
        assert np.array_equal(a.vloss.view(np.int64), b.vloss.view(np.int64))
    if a.ids is not None and b.ids is not None:
        assert list(a.ids) == list(b.ids)


def test_shipped_topology_matches_fixture_and_reader():
    path = os.path.join(DATA, "topology.graphml.xml.xz")
    nat = parse_graphml(path)
    assert nat.n == 183 and nat.m == 16836 and not nat.directed
    same(nat, read_graphml(path))
    fix = Topology.load_npz(os.path.join(GOLDEN, "shipped_topology.npz"))
    same(nat, fix)


def test_doc_example():
    xml = open(os.path.join(DATA, "doc_example.graphml")).read()
    same(parse_graphml(xml), read_graphml(xml))


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_roundtrip_random(seed):
    top = G.random_sparse(300, 5, seed=seed)
    xml = write_graphml(top)
    nat = parse_graphml(xml)
    same(nat, read_graphml(xml))
    assert np.array_equal(nat.latency, top.latency) and np.array_equal(nat.loss, top.loss)


HEAD = ('<?xml version="1.0"?>\n<!-- comment -->\n'
        '<graphml xmlns="http://graphml.graphdrawing.org/xmlns">\n')


def test_defaults_missing_values_and_forward_edges():
    xml = HEAD + '''
  <key id="l" for="edge" attr.name="latency" attr.type="double"><default>7.5</default></key>
  <key id="p" for="edge" attr.name="packetloss" attr.type="double"/>
  <key id="v" for="node" attr.name="packetloss" attr.type="double"><default>0.25</default></key>
  <key id="g" for="graph" attr.name="preferdirectpaths" attr.type="string"/>
  <graph edgedefault="directed">
    <data key="g">Yes please</data>
    <edge source="b" target="a&amp;1"><data key="p">0.5</data></edge>
    <node id="a&amp;1"/>
    <node id="b"><data key="v">0.125</data></node>
    <?pi ignored?>
    <edge source="a&amp;1" target="b"><data key="l"> 1e-3 </data><data key="p"/></edge>
    <edge source="b" target="b"><data key="l">not-a-number</data><data key="p"><![CDATA[0.75]]></data></edge>
  </graph>
</graphml>'''
    nat = parse_graphml(xml)
    same(nat, read_graphml(xml))
    assert nat.directed and nat.prefers_direct and nat.ids == ["a&1", "b"]
    assert list(nat.src) == [1, 0, 1] and list(nat.dst) == [0, 1, 1]
    assert nat.latency[0] == 7.5 and nat.latency[1] == 1e-3 and np.isnan(nat.latency[2])
    assert nat.loss[0] == 0.5 and np.isnan(nat.loss[1]) and nat.loss[2] == 0.75
    assert list(nat.vloss) == [0.25, 0.125]


@pytest.mark.parametrize("val,expect", [("true", True), ("TRUE", True), ("1", True),
                                        ("yes", True), ("false", False), ("", False),
                                        ("no", False),
                                        ("  yes", False)])   # no strip: g_ascii_strncasecmp, topology.c:772
def test_prefers_direct_values(val, expect):
    xml = HEAD + ('<key id="g" for="graph" attr.name="preferdirectpaths" attr.type="string"/>'
                  '<graph edgedefault="undirected"><data key="g">%s</data>'
                  '<node id="x"/></graph></graphml>' % val)
    nat = parse_graphml(xml)
    assert nat.prefers_direct is expect
    assert nat.prefers_direct == read_graphml(xml).prefers_direct
    assert nat.vloss is None and not nat.directed and nat.m == 0


@pytest.mark.parametrize("bad", [
    '<graph><node id="a"/><node id="a"/></graph></graphml>',          # duplicate id
    '<graph><node id="a"/><edge source="a" target="zz"/></graph></graphml>',   # unknown node
    '<graph><node id="a"></graph></graphml>',                          # bad nesting
    '<graph><node id="a"/>',                                           # truncated
    '<node id="a"/></graphml>',                                        # no graph
])
def test_malformed_rejected(bad):
    with pytest.raises(EngineError):
        parse_graphml(HEAD + bad)
