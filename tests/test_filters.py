"""CPU: metadata filter semantics and the row-mask layout rfx_search_masked reads (rfx.filters)."""
import numpy as np
import pytest

from rfx import filters


def test_normalize_metadata_forms():
    gem = [{"key": "tenant", "string_value": "acme"}, {"key": "year", "numeric_value": 2024},
           {"key": "bad"}, {"nokey": 1}, {"key": " ", "string_value": "x"}]
    assert filters.normalize_metadata(gem) == {"tenant": "acme", "year": 2024}
    assert filters.normalize_metadata({"a": 1, "b": [1]}) == {"a": 1}
    assert filters.normalize_metadata(None) == {}


@pytest.mark.parametrize("md,filt,ok", [
    ({"t": "a"}, {"t": "a"}, True),
    ({"t": "a"}, {"t": "A"}, False),
    ({"t": "a"}, {"t": ["b", "a"]}, True),
    ({"t": "a", "y": 3}, {"t": "a", "y": 3.0}, True),
    ({"t": "a", "y": 3}, {"t": "a", "y": 4}, False),
    ({"t": "a"}, {"u": "a"}, False),
    ({"f": True}, {"f": 1}, False),
    ({"f": 1}, {"f": True}, False),
    ({"f": True}, {"f": [False, True]}, True),
    ({"n": "3"}, {"n": 3}, False),
])
def test_file_matches(md, filt, ok):
    assert filters.file_matches(md, filt) is ok


def test_check_filter():
    assert filters.check_filter(None) is None and filters.check_filter({}) is None
    assert filters.check_filter({" t ": "a"}) == {"t": "a"}
    for bad in ("t=a", {"": 1}, {"t": []}, {"t": {"x": 1}}, {"t": [1, None]}):
        with pytest.raises(ValueError):
            filters.check_filter(bad)
    assert filters.filter_key({"b": 1, "a": [2]}) == filters.filter_key({"a": [2], "b": 1})


def test_row_mask_words_layout():
    words = filters.row_mask_words(100, [(0, 3), (31, 2), (64, 1), (99, 1)])
    assert words.dtype == np.int32 and words.shape == (4,)
    bits = np.unpackbits(words.view(np.uint8), bitorder="little")
    assert set(np.flatnonzero(bits)) == {0, 1, 2, 31, 32, 64, 99}
    assert filters.row_mask_words(0, []).shape == (1,)
