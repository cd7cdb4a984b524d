"""Host-side logic of the drop-in LearnedIndex (no GPU): the caller-visible
`data_navigation['category'] = pred_categories` side effect of search()
(LearnedIndex.py:67) and when an attached caller may skip rewriting it."""
import numpy as np
import pandas as pd

from li.LearnedIndex import LearnedIndex


def _frame(n=1000):
    d = pd.DataFrame(np.random.default_rng(0).random((n, 4)).astype(np.float32))
    d.index += 1
    return d


def test_category_written_without_attach():
    li = LearnedIndex()
    d = _frame()
    lab = np.arange(1000) % 7
    li._set_category(d, lab)
    assert np.array_equal(d["category"].to_numpy(), lab)
    assert li._cat_written is None            # not attached: every call writes
    d["category"] = 0
    li._set_category(d, lab)
    assert np.array_equal(d["category"].to_numpy(), lab)


def test_attached_rewrite_skipped_only_when_unchanged():
    li = LearnedIndex()
    d = _frame()
    lab = np.arange(1000) % 7
    li._trusted = ("attached", None)          # as after attach(d, ..., lab)
    li._attached_labels = lab
    li._set_category(d, lab)
    assert np.array_equal(d["category"].to_numpy(), lab)
    first = li._cat_written
    assert first is not None
    li._set_category(d, lab)                  # the same objects, column untouched: skipped
    assert li._cat_written == first
    assert np.array_equal(d["category"].to_numpy(), lab)
    d["category"] = np.zeros(1000, np.int64)  # the caller replaced the column
    li._set_category(d, lab)
    assert np.array_equal(d["category"].to_numpy(), lab)
    other = lab.copy()                        # other labels: written
    other[0] = 6
    li._set_category(d, other)
    assert np.array_equal(d["category"].to_numpy(), other)
    li.detach()
    assert li._cat_written is None


def test_attached_index_served_only_for_the_attached_objects():
    """The trust of attach(): the cached HBM index is served
    without a content hash only for the very objects attached -- held by
    strong references, so a new frame cannot inherit a freed one's id() or
    buffer address -- and only while their value arrays are where they were."""
    li = LearnedIndex()
    nav, ds = _frame(), _frame()
    lab = np.arange(1000) % 7
    li._index, li._cache_key = object(), ("key",)
    li._trusted = (li._identity(nav, ds, lab), li._cache_key, (ds, lab, nav.index))
    assert li._is_attached(nav, ds, lab)
    assert not li._is_attached(nav, ds.copy(), lab)          # equal values, another object
    assert not li._is_attached(nav, ds, lab.copy())
    nav2 = nav.copy()
    assert not li._is_attached(nav2, ds, lab)                # another index object
    li._cache_key = ("other",)                               # the cache was rebuilt
    assert not li._is_attached(nav, ds, lab)
    li._cache_key = ("key",)
    ds[4] = 1.0                                              # a new column: new value arrays
    assert not li._is_attached(nav, ds, lab)
    # the trust holds the objects alive: dropping the caller's names frees nothing
    import weakref
    r = weakref.ref(lab)
    del lab
    assert r() is not None
    li.detach()
    assert li._trusted is None
