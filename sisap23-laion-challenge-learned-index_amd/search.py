"""CLI drop-in for the reference's search/search.py on MI355X.

Same flags and defaults (search.py:169-248), same flow (search.py:23-166):
load pca96 + clip768 H5 data, normalise pca96 (preprocess), build the index,
then for every bucket count time `li.search` (R > 1) or `li.search_single`
(R == 1) exactly over the span search.py:116-141 and write the H5 result file
result/{kind}/{size}/learned-index-...h5 (utils.py:85-97) read by eval/.

Differences: the data must already be under data/ (no network here), and
`--synthetic N` runs the same flow on an N-row synthetic clip768-like set.

`--gpus N` (an addition) shards the index over N GPUs of one node: without a
launcher the script starts its own N rank processes before any GPU call
(li.dist.launch_ranks; under torchrun it runs as one of the ranks).  Every
rank loads the same files and runs the same flow; li.LearnedIndex's
process-group mode builds one stripe of every bucket per rank and returns the
whole answer on every rank; rank 0 writes the H5 file.  The results are
bitwise those of one GPU.
"""
import argparse
import logging
import os
import sys
import time

import numpy as np
import pandas as pd

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from li.LearnedIndex import LearnedIndex  # noqa: E402
from li.model import data_X_to_torch  # noqa: E402
from li.utils import prepare, save_as_pickle, store_results  # noqa: E402

np.random.seed(2023)
logging.basicConfig(level=logging.INFO,
                    format='[%(asctime)s][%(levelname)-5.5s][%(name)-.20s] %(message)s')
LOG = logging.getLogger(__name__)


def _normalize(x):
    """sklearn.preprocessing.normalize(x) (norm='l2', axis=1, dense), the
    call at search.py:50-52, restated from sklearn 1.x (_data.normalize,
    extmath.row_norms, _handle_zeros_in_scale): float16 / float32 / float64
    input keeps its dtype (other dtypes become float64), norms by einsum in
    that dtype, norms < 10 * eps(dtype) replaced by 1, rows divided in place."""
    x = np.array(x, copy=True)
    if x.dtype not in (np.float16, np.float32, np.float64):
        x = x.astype(np.float64)
    n = np.sqrt(np.einsum("ij,ij->i", x, x))
    n[n < 10 * np.finfo(n.dtype).eps] = 1.0
    x /= n[:, None]
    return x


def _load(kind, size, key):
    """search.py:48-49 / :79-87 (np.array(h5py.File(...)[key])) on liblmi_h5.so."""
    from li import h5
    data = h5.read_dataset(os.path.join("data", kind, size, "dataset.h5"), key)
    queries = h5.read_dataset(os.path.join("data", kind, size, "query.h5"), key)
    return data, queries


def _synthetic(n, nq=10_000):
    from li import synth
    x, cen = synth.np_mixture(n, 768, 400, 2023)
    q, _ = synth.np_mixture(nq, 768, 400, 4242, centres=cen)
    P = synth.np_projection(768, 96, 96)
    return x @ P, q @ P, x, q


def run(kind, key, size='100K', k=10, index_type='learned-index', n_buckets_perc=None,
        n_categories=None, epochs=100, model_type='MLP', lr=0.1, preprocess=False, save=False,
        synthetic=0, semantics='reference', index_path=None):
    rank, world = 0, 1
    if int(os.environ.get("WORLD_SIZE", "1")) > 1:
        # one rank of `--gpus N` / torchrun: the process group (and this
        # rank's GPU) first, before the router or the index touch a device
        from li.dist import init_from_env
        rank, world, _ = init_from_env()
        if rank:
            logging.getLogger().setLevel(logging.WARNING)
    n_buckets_perc = [int((b / 100) * n_categories) for b in n_buckets_perc]   # search.py:37-38
    n_buckets_perc = list(set([b for b in n_buckets_perc if b > 0]))
    LOG.info(f'Running with: kind={kind}, key={key}, size={size}, n_buckets_perc={n_buckets_perc}, '
             f'n_categories={n_categories}, epochs={epochs}, lr={lr}, model_type={model_type}, '
             f'preprocess={preprocess}, save={save}')
    if synthetic:
        data, queries, data_search, queries_search = _synthetic(synthetic)
    else:
        prepare(kind, size)
        data, queries = _load(kind, size, key)
    if preprocess:
        data, queries = _normalize(data), _normalize(queries)
    if index_type != 'learned-index':
        raise Exception(f'Unknown index type: {index_type}')
    s = time.time()
    data = pd.DataFrame(data)
    data.index += 1
    if not synthetic:
        kind_search, key_search = 'clip768v2', 'emb'
        if kind != kind_search:
            prepare(kind_search, size)
            data_search, queries_search = _load(kind_search, size, key_search)
        else:
            data_search, queries_search = data.values, queries
    data_search = pd.DataFrame(data_search)
    data_search.index += 1
    if index_path:
        # a pickled index (the reference's own save_as_pickle format, row f1):
        # its router labels the data as build() would (LearnedIndex.py:240)
        from li.index_io import load_index, object_labels
        t0 = time.time()
        li = load_index(index_path)
        pred_categories = object_labels(li, data)
        build_t = time.time() - t0
    else:
        li = LearnedIndex()
        pred_categories, build_t = li.build(data, n_categories=n_categories, epochs=epochs, lr=lr)
    LOG.info(f'Pure build time: {build_t}')
    LOG.info(f'Overall build time: {time.time() - s}')
    # the bucket-sorted corpus goes to HBM here, before the timed loop, and
    # the frames are trusted from now on (this flow never changes them), so
    # no timed call re-hashes 15 GB of clip768 (LearnedIndex.attach)
    if os.environ.get("LMI_NO_ATTACH") != "1":   # (diagnostic: hash-checked calls instead)
        li.attach(data, data_search, pred_categories)
    if save:
        os.makedirs('./models', exist_ok=True)
        save_as_pickle(f'./models/{kind}-{size}-ep={epochs}-lr={lr}-cat={n_categories}'
                       f'-model={model_type}-prep={preprocess}.pkl', li)
    for bucket in n_buckets_perc:
        if world > 1:
            # the ranks enter the timed span together, so rank 0's clock is
            # the job's (each call ends in collectives every rank joins)
            import torch.distributed as dist
            dist.barrier()
        s = time.time()
        LOG.info(f'Searching with {bucket} buckets')
        if bucket > 1:
            dists, nns = li.search(data_navigation=data, queries_navigation=queries,
                                   data_search=data_search, queries_search=queries_search,
                                   pred_categories=pred_categories, n_buckets=bucket, k=k,
                                   use_threshold=True, semantics=semantics)
        else:
            _, pred_proba_categories = li.model.predict_proba(data_X_to_torch(queries))
            data['category'] = pred_categories
            dists, nns = li.search_single(data_navigation=data, data_search=data_search,
                                          queries_search=queries_search,
                                          pred_categories=pred_proba_categories[:, 0], k=k)
        search_t = time.time() - s
        LOG.info(f'Search time: {search_t}')
        short_identifier = 'learned-index'
        identifier = (f'{short_identifier}-{kind}-{size}-ep={epochs}-lr={lr}-cat='
                      f'{n_categories}-model={model_type}-buck={bucket}')
        store_results(os.path.join("result/", kind, size, f"{identifier}.h5"),
                      short_identifier.capitalize(), kind, dists, nns, build_t, search_t,
                      identifier, size)


if __name__ == "__main__":
    from li.dist import gpus_arg, launch_ranks
    if gpus_arg(sys.argv[1:]) > 1 and "WORLD_SIZE" not in os.environ:
        # before anything touches a GPU: the ranks are child processes
        sys.exit(launch_ranks(gpus_arg(sys.argv[1:]), sys.argv[1:], os.path.abspath(__file__),
                              relay_stdout=False))
    parser = argparse.ArgumentParser()
    parser.add_argument("--dataset", default="pca96v2")
    parser.add_argument("--emb", default="pca96")
    parser.add_argument("--size", default="10M")
    parser.add_argument("--k", default=10, type=int)
    parser.add_argument("--n-categories", default=122, type=int,
                        help='Number of categories (= buckets) to create')
    parser.add_argument("--epochs", default=205, type=int, help='Number of epochs to train the model for')
    parser.add_argument("--model-type", default='MLP-5', type=str, help='Model type to use for the learned index')
    parser.add_argument("--lr", default=0.009, type=float, help='Learning rate')
    parser.add_argument('-bp', '--buckets-perc', nargs='+', default=[4],
                        help='Percentage of the most similar buckets to look for the candidate answer in')
    parser.add_argument("--preprocess", default=True, type=bool, help='Whether to normalize the data or not')
    parser.add_argument("--save", default=False, type=bool, help='Whether to save the model or not')
    parser.add_argument("--synthetic", default=0, type=int,
                        help='run on N synthetic rows instead of data/ (this build has no network)')
    parser.add_argument("--semantics", default="reference", choices=["reference", "exact"],
                        help='reference: LearnedIndex.search round merge (default); exact: exact '
                             'top-k over the probed buckets')
    parser.add_argument("--gpus", default=1, type=int,
                        help='shard the index over N GPUs of this node (one process per GPU, '
                             'started by this script unless a launcher set WORLD_SIZE)')
    parser.add_argument("--index", default=None,
                        help='load a pickled LearnedIndex (save_as_pickle format) instead of '
                             'building one; its router labels the data')
    args = parser.parse_args()
    assert args.size in ['100K', '300K', '10M', '30M', '100M']
    run(args.dataset, args.emb, args.size, args.k, 'learned-index',
        [int(b) for b in args.buckets_perc], args.n_categories, args.epochs, args.model_type,
        args.lr, args.preprocess, args.save, synthetic=args.synthetic, semantics=args.semantics,
        index_path=args.index)
