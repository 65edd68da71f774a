"""merged_passes' unit mapping (host logic, no GPU): the tuner's destination-
group candidates set merge_unit "group", which names group_passes' cache entry;
a propagate_overlapped layer sharing the graph (GIN max / SAGE after a fused
GIN layer tuned to "group") must merge the plan's steps instead of reading
that entry (test_sharded_gin_sage_layers hit it when the tuner chose "group")."""

from keras_geometric_amd import distributed as kd


def test_merge_unit_maps_group_to_step():
    assert kd._merge_unit("group") == "step"
    for u in ("step", "chunk", "none"):
        assert kd._merge_unit(u) == u


def test_prune_pulls_switch(monkeypatch):
    monkeypatch.delenv("KGX_HALO_PRUNE", raising=False)
    assert kd.prune_pulls()
    monkeypatch.setenv("KGX_HALO_PRUNE", "0")
    assert not kd.prune_pulls()
