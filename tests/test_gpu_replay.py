"""The device replay (lmi_replay_device) against its host twin (lmi_replay,
itself pinned to the reference's outputs by test_oracle_golden.py): bit for
bit on random lists that drive every branch — thresholds, the <k quirk of
thresholded rounds and of tiny buckets, empty groups, fillers, ties, R == 1
with and without threshold_dist, k_final > k_round."""
import numpy as np
import pytest
import torch

import lmi_oracle as O
import workloads
from li.index import replay, replay_device

pytestmark = pytest.mark.gpu


def _random_lists(seed, nq, R, C, kl, tiny=(), empty=(), probe_empty=False):
    rng = np.random.default_rng(seed)
    size = rng.integers(40, 400, C).astype(np.int64)
    for c in tiny:
        size[c] = rng.integers(1, kl)
    for c in empty:
        size[c] = 0
    off = np.concatenate([[0], np.cumsum(size)])
    # probe_empty: the router may rank a category without objects among a
    # query's top R (a group the reference's groupby never visits)
    live = np.arange(C) if probe_empty else np.nonzero(size > 0)[0]
    p = rng.dirichlet(np.full(live.size, 0.5))
    classes = np.stack([rng.choice(live, R, replace=False, p=p) for _ in range(nq)]).astype(np.int32)
    d = np.full((nq, R, kl), np.inf, np.float32)
    pos = np.full((nq, R, kl), -1, np.int32)
    for q in range(nq):
        for r in range(R):
            c = classes[q, r]
            n = min(kl, size[c])
            pp = rng.choice(size[c], n, replace=False) + off[c]
            dd = np.round(rng.random(n) * 0.6 + 0.2, 3).astype(np.float32)  # ties likely
            o = np.lexsort((pp, dd))
            d[q, r, :n], pos[q, r, :n] = dd[o], pp[o]
    ids = rng.permutation(int(off[-1])).astype(np.int64) + 1
    return classes, d, pos, size, ids


@pytest.mark.parametrize("seed", range(8))
@pytest.mark.parametrize("use_threshold", [True, False])
def test_device_replay_equals_host_replay(seed, use_threshold):
    R = 1 + seed % 4
    classes, d, pos, size, ids = _random_lists(seed, nq=700, R=R, C=24, kl=10, tiny=(3, 7),
                                               empty=(5, 11), probe_empty=seed >= 4)
    for k_final in ([10] if R == 1 else [10, 14]):
        if R > 1 and k_final > 10 * R:
            continue
        ref_d, ref_a = replay(classes, d, pos, k_round=10, k_final=k_final, bucket_size=size,
                              pos_to_id=ids, use_threshold=use_threshold)
        dev = torch.device("cuda")
        dd, aa, st = replay_device(torch.from_numpy(classes).to(dev), torch.from_numpy(d).to(dev),
                                   torch.from_numpy(pos).to(dev), k_round=10, k_final=k_final,
                                   bucket_size=torch.from_numpy(size).to(dev),
                                   pos_to_id=torch.from_numpy(ids).to(dev),
                                   use_threshold=use_threshold)
        assert int(st.item()) == 0
        np.testing.assert_array_equal(dd.cpu().numpy(), ref_d)
        np.testing.assert_array_equal(aa.cpu().numpy().view(np.uint32), ref_a)


def test_device_replay_single_with_threshold():
    classes, d, pos, size, ids = _random_lists(11, nq=500, R=1, C=16, kl=10, tiny=(2,))
    thr = np.random.default_rng(3).random(500) * 0.5 + 0.3
    ref_d, ref_a = replay(classes, d, pos, k_round=10, k_final=10, bucket_size=size, pos_to_id=ids,
                          use_threshold=False, thr_round0=thr)
    dev = torch.device("cuda")
    dd, aa, st = replay_device(torch.from_numpy(classes).to(dev), torch.from_numpy(d).to(dev),
                               torch.from_numpy(pos).to(dev), k_round=10, k_final=10,
                               bucket_size=torch.from_numpy(size).to(dev),
                               pos_to_id=torch.from_numpy(ids).to(dev), use_threshold=False,
                               thr_round0=torch.from_numpy(thr).to(dev))
    assert int(st.item()) == 0
    np.testing.assert_array_equal(dd.cpu().numpy(), ref_d)
    np.testing.assert_array_equal(aa.cpu().numpy().view(np.uint32), ref_a)


@pytest.mark.parametrize("seed", [5, 7])
def test_device_replay_on_real_lists_reaches_every_branch(seed):
    """Oracle lists of the golden-style skewed workload (quirk0, quirk_thr,
    skipped groups and fillers all occur) through both replays."""
    w = workloads.clustered(n=4000, nq=300, C=16, seed=seed, label_mode="skewed")
    classes = O.rank_classes(O.mlp_forward(w["qn"], w["layers"]))[:, :4].astype(np.int32)
    order, off = O.layout(w["labels"], 16)
    lists_d, lists_p = O.bucket_lists(w["labels"], w["x"], w["q"], classes, 4, 10, 16)
    st = {}
    O.replay(classes, lists_d, lists_p, k_round=10, k_final=10, bucket_size=np.diff(off),
             pos_to_id=np.arange(1, 4001)[order], use_threshold=True, stats=st)
    assert st["quirk0"] > 0 and st["quirk_thr"] > 0 and st["skipped"] > 0 and st["fillers"] > 0
    ids = np.arange(1, 4001)[order]
    ref_d, ref_a = replay(classes, lists_d, lists_p, k_round=10, k_final=10,
                          bucket_size=np.diff(off), pos_to_id=ids, use_threshold=True)
    dev = torch.device("cuda")
    dd, aa, s2 = replay_device(torch.from_numpy(classes).to(dev), torch.from_numpy(lists_d).to(dev),
                               torch.from_numpy(lists_p.astype(np.int32)).to(dev), k_round=10,
                               k_final=10, bucket_size=torch.from_numpy(np.diff(off)).to(dev),
                               pos_to_id=torch.from_numpy(ids).to(dev), use_threshold=True)
    assert int(s2.item()) == 0
    np.testing.assert_array_equal(dd.cpu().numpy(), ref_d)
    np.testing.assert_array_equal(aa.cpu().numpy().view(np.uint32), ref_a)


@pytest.mark.parametrize("use_threshold", [True, False])
@pytest.mark.parametrize("nq,C", [(6000, 5), (2500, 4), (12000, 3)])
def test_device_replay_large_groups(use_threshold, nq, C):
    """Groups whose relevant positions exceed the kernel's LDS staging
    (kUCap = 8192 entries) take the global-scratch path; small ones in the
    same launch stay in LDS.  Selection runs from registers up to 16384
    entries (thresholded rounds of nq=2500, C=4: 9.4K-14.4K), from the
    global share beyond (nq=6000, C=5: 19K-25K; nq=12000, C=3: up to 74K)."""
    classes, d, pos, size, ids = _random_lists(21, nq=nq, R=3, C=C, kl=10, tiny=(C - 1,))
    ref_d, ref_a = replay(classes, d, pos, k_round=10, k_final=10, bucket_size=size,
                          pos_to_id=ids, use_threshold=use_threshold)
    assert np.bincount(classes[:, 1], minlength=C).max() * 10 > 8192
    dev = torch.device("cuda")
    dd, aa, st = replay_device(torch.from_numpy(classes).to(dev), torch.from_numpy(d).to(dev),
                               torch.from_numpy(pos).to(dev), k_round=10, k_final=10,
                               bucket_size=torch.from_numpy(size).to(dev),
                               pos_to_id=torch.from_numpy(ids).to(dev), use_threshold=use_threshold)
    assert int(st.item()) == 0
    np.testing.assert_array_equal(dd.cpu().numpy(), ref_d)
    np.testing.assert_array_equal(aa.cpu().numpy().view(np.uint32), ref_a)


@pytest.mark.parametrize("use_threshold", [True, False])
def test_device_replay_wide_position_range(use_threshold):
    """A bucket of 300K rows: a group's relevant positions can span more than
    the group kernel's selection bitmap (192K positions), so that group
    selects by wave-minimum rounds; the other buckets take the bitmap."""
    rng = np.random.default_rng(77)
    nq, R, kl = 400, 2, 10
    size = np.array([300_000, 60, 250, 7], np.int64)
    off = np.concatenate([[0], np.cumsum(size)])
    classes = np.stack([rng.choice(4, R, replace=False, p=[0.5, 0.2, 0.2, 0.1])
                        for _ in range(nq)]).astype(np.int32)
    d = np.full((nq, R, kl), np.inf, np.float32)
    pos = np.full((nq, R, kl), -1, np.int32)
    for q in range(nq):
        for r in range(R):
            c = classes[q, r]
            n = min(kl, int(size[c]))
            pp = np.unique(rng.integers(0, size[c], 4 * n))[:n]
            pp = rng.permutation(pp)[:n] + off[c]
            dd = np.round(rng.random(pp.size) * 0.6 + 0.2, 3).astype(np.float32)
            o = np.lexsort((pp, dd))
            d[q, r, :pp.size], pos[q, r, :pp.size] = dd[o], pp[o]
    ids = rng.permutation(int(off[-1])).astype(np.int64) + 1
    ref_d, ref_a = replay(classes, d, pos, k_round=10, k_final=10, bucket_size=size, pos_to_id=ids,
                          use_threshold=use_threshold)
    dev = torch.device("cuda")
    dd_, aa, st = replay_device(torch.from_numpy(classes).to(dev), torch.from_numpy(d).to(dev),
                                torch.from_numpy(pos).to(dev), k_round=10, k_final=10,
                                bucket_size=torch.from_numpy(size).to(dev),
                                pos_to_id=torch.from_numpy(ids).to(dev), use_threshold=use_threshold)
    assert int(st.item()) == 0
    np.testing.assert_array_equal(dd_.cpu().numpy(), ref_d)
    np.testing.assert_array_equal(aa.cpu().numpy().view(np.uint32), ref_a)


@pytest.mark.parametrize("k_final,R", [(10, 4), (14, 3), (10, 1)])
def test_phased_replay_equals_one_call(k_final, R):
    """lmi_replay_device_phase: GROUPS (the classes only; zeroes the status
    word) then ROUNDS on one workspace = the one-call replay = the host
    replay, bit for bit (R = 1, k_final = k_round and k_final > k_round)."""
    from li import _lib
    classes, d, pos, size, ids = _random_lists(31 + R, nq=500, R=R, C=24, kl=10, tiny=(3,),
                                               empty=(5,))
    dev = torch.device("cuda")
    T = lambda a: torch.from_numpy(a).to(dev)  # noqa: E731
    kw = dict(k_round=10, k_final=k_final, bucket_size=T(size), pos_to_id=T(ids), use_threshold=True)
    one = replay_device(T(classes), T(d), T(pos), **kw)
    ws = torch.empty(1 << 24, dtype=torch.uint8, device=dev)
    w = 10 if R == 1 else k_final
    out = (torch.empty((500, w), dtype=torch.float64, device=dev),
           torch.empty((500, w), dtype=torch.int32, device=dev),
           torch.full((1,), 0x70, dtype=torch.int32, device=dev))
    replay_device(T(classes), None, None, out=out, phases=_lib.LMI_REPLAY_PHASE_GROUPS, ws=ws, k_list=10, **kw)
    torch.cuda.synchronize()
    assert int(out[2].item()) == 0
    replay_device(T(classes), T(d), T(pos), out=out, phases=_lib.LMI_REPLAY_PHASE_ROUNDS, ws=ws, **kw)
    assert torch.equal(out[0], one[0]) and torch.equal(out[1], one[1]) and int(out[2].item()) == 0
    ref_d, ref_a = replay(classes, d, pos, k_round=10, k_final=k_final, bucket_size=size, pos_to_id=ids,
                          use_threshold=True)
    np.testing.assert_array_equal(out[0].cpu().numpy(), ref_d)
    np.testing.assert_array_equal(out[1].cpu().numpy().view(np.uint32), ref_a)
