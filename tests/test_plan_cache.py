"""The engine's plan cache is bounded (CPU): a shape is cached on its second sighting, entries
and workspace bytes are capped (least recently used out), clear() empties it."""
from kvcompress._engine import _PlanCache


def test_second_sighting_and_bounds():
    c = _PlanCache(capacity=3, max_bytes=1000, seen_capacity=4)
    assert not c.admit("a")          # first sighting: not cached
    assert c.admit("a")              # second: cache it
    c.put("a", ("plan-a",), 400)
    assert c.get("a")[0] == "plan-a" and c.bytes == 400
    for key in ("b", "c"):
        c.admit(key)
        assert c.admit(key)
        c.put(key, (key,), 400)
    assert "a" not in c.entries      # 1200 > 1000 bytes: the oldest went
    assert set(c.entries) == {"b", "c"} and c.bytes == 800
    c.get("b")                       # b most recently used
    c.put("d", ("d",), 300)
    assert set(c.entries) == {"b", "d"} and c.bytes == 700
    c.put("huge", ("h",), 5000)      # larger than the cap: never cached
    assert "huge" not in c.entries
    for key in "pqrstu":             # the sightings table is bounded too
        c.admit(key)
    assert len(c.seen) == 4
    c.clear()
    assert not c.entries and not c.seen and c.bytes == 0
