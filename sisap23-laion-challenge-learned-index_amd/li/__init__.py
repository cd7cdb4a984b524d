"""li — MI355X-native drop-in for the reference's `li` package (search hot path).

Module map (reference file -> here):
  search/li/LearnedIndex.py -> li/LearnedIndex.py  (search / search_single on the GPU)
  search/li/model.py        -> li/model.py         (Model, NeuralNetwork.predict[_proba] on K1)
  search/li/utils.py        -> li/utils.py         (distance helpers, store_results)
  search/li/Baseline.py     -> li/Baseline.py
  search/li/Logger.py       -> li/Logger.py
New: li/index.py (device index + pipeline), li/_lib.py (C-ABI binding),
li/dist.py (multi-GPU stripes + RCCL), li/synth.py (synthetic workloads).
"""
__version__ = "0.1.0"
