"""Pin the CPU oracle against the reference's own SnapshotV1 golden vectors.

tests/golden/v1/*.json are the data files of packages/dds/sequence/src/test/snapshots/v1/, produced
by generateSharedStrings.ts:24-98 and compared with deepStrictEqual in snapshotVersion.spec.ts:198-212.
Here the same local (non-collaborative) edit sequences are replayed on the oracle and its SnapshotV1
blobs must equal the fixture blobs byte for byte.
"""
import json
import os

import pytest

from oracle import OracleDoc

GOLDEN = os.path.join(os.path.dirname(__file__), "golden", "v1")
SIZE_OF_FIRST_CHUNK = 10000  # snapshotlegacy.ts:56
INSERT_TEXT = "text"


def build_doc(name):
    """generateSharedStrings.ts:24-98, the v1 entries."""
    d = OracleDoc(observer=None)
    if name == "headerOnly":
        for i in range(SIZE_OF_FIRST_CHUNK // len(INSERT_TEXT) // 2):
            d.insert_text_local(0, f"{INSERT_TEXT}{i}")
    elif name in ("headerAndBody", "withMarkers", "withAnnotations"):
        for i in range(SIZE_OF_FIRST_CHUNK // len(INSERT_TEXT) * 2):
            d.insert_text_local(0, f"{INSERT_TEXT}{i}")
        if name == "withMarkers":
            i = 0
            while i < d.length():
                props = {"ItemType": "Paragraph", "Properties": {"Bold": False}, "markerId": f"marker{i}",
                         "referenceTileLabels": ["Eop"]}
                d.insert_marker_local(i, 1, json.dumps(props))
                i += 70
        if name == "withAnnotations":
            i = 0
            while i < d.length():
                d.annotate_local(i, i + 10, json.dumps({"bold": True}))
                i += 70
    elif name == "largeBody":
        for i in range(SIZE_OF_FIRST_CHUNK):
            d.insert_text_local(0, f"{INSERT_TEXT}-{i}")
    return d


def fixture_blobs(name):
    with open(os.path.join(GOLDEN, name + ".json")) as f:
        tree = json.load(f)
    content = [e for e in tree["entries"] if e["path"] == "content"][0]
    return [(e["path"], e["value"]["contents"]) for e in content["value"]["entries"]]


@pytest.mark.parametrize("name", ["headerOnly", "headerAndBody", "largeBody", "withMarkers", "withAnnotations"])
def test_snapshot_v1_fixture(name):
    d = build_doc(name)
    tree = json.loads(d.snapshot_json())
    got = [(e["path"], e["value"]["contents"]) for e in tree["entries"]]
    want = fixture_blobs(name)
    assert [p for p, _ in got] == [p for p, _ in want]
    for (p, g), (_, w) in zip(got, want):
        assert g == w, f"blob {p} differs"


# generateSharedStrings.ts:14-22: "legacy" writes the catch-up blob under the option's name,
# "legacyWithCatchUp" under the default "catchupOps"; both with the legacy (default) snapshot format
LEGACY_CATCHUP = {"legacy": "randomNameForCatchUpOps", "legacyWithCatchUp": "catchupOps"}


def legacy_fixture_blobs(version, name):
    with open(os.path.join(os.path.dirname(__file__), "golden", version, name + ".json")) as f:
        tree = json.load(f)
    content = [e for e in tree["entries"] if e["path"] == "content"][0]
    return [(e["path"], e["value"]["contents"]) for e in content["value"]["entries"]]


@pytest.mark.parametrize("version", sorted(LEGACY_CATCHUP))
@pytest.mark.parametrize("name", ["headerOnly", "headerAndBody", "largeBody", "withMarkers", "withAnnotations"])
def test_snapshot_legacy_fixture(version, name):
    """SnapshotLegacy (snapshotlegacy.ts:103-238) bytes of the same documents equal the legacy fixtures."""
    d = build_doc(name)
    tree = json.loads(d.snapshot_legacy_json(catch_up_name=LEGACY_CATCHUP[version]))
    got = [(e["path"], e["value"]["contents"]) for e in tree["entries"]]
    want = legacy_fixture_blobs(version, name)
    assert [p for p, _ in got] == [p for p, _ in want]
    for (p, g), (_, w) in zip(got, want):
        assert g == w, f"blob {p} differs"
