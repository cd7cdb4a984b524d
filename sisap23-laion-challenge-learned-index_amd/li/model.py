"""Drop-in for the reference's search/li/model.py with inference on K1.

Same names, architectures and return types as the reference:

  Model            model.py:15-83   nn.Sequential 'layers' of Linear/ReLU per
                                     model_type ('MLP' ... 'MLP-9')
  data_X_to_torch  model.py:86-89
  data_to_torch    model.py:92-96
  get_device       model.py:99-111
  NeuralNetwork    model.py:114-229  train / train_batch unchanged (torch;
                                     index build is outside the hot path),
                                     predict / predict_proba on the GPU router
                                     kernel (lmi_router, liblmi_hip.so)
  LIDataset        model.py:232-240  (1-based __getitem__, as the reference)

predict_proba returns (probs f32 ndarray, classes int64 ndarray), both
(n, n_classes), classes by descending probability (ties to the lower class),
like `softmax(outputs, dim=1).topk(C)` (model.py:220-227).  predict returns
argmax labels (int64), like `torch.max(outputs, 1)` (model.py:207-211).
There is no CPU fallback: on a host without a HIP device these raise.
"""
from __future__ import annotations

from typing import Tuple

import numpy as np
import torch
import torch.utils.data

from .Logger import Logger

torch.manual_seed(2023)
np.random.seed(2023)

_ARCH = {
    "MLP": (128,), "MLP-2": (64,), "MLP-3": (256,), "MLP-4": (512,), "MLP-5": (256, 128),
    "MLP-6": (32,), "MLP-7": (16,), "MLP-8": (8,),
}


class Model(torch.nn.Module):
    """The model class representing the index (model.py:15-83)."""

    def __init__(self, input_dim=768, output_dim=1000, model_type=None):
        super().__init__()
        if model_type in _ARCH:
            dims = [input_dim, *_ARCH[model_type], output_dim]
            mods = []
            for i, (a, b) in enumerate(zip(dims, dims[1:])):
                mods.append(torch.nn.Linear(a, b))
                if i + 2 < len(dims):
                    mods.append(torch.nn.ReLU())
            self.layers = torch.nn.Sequential(*mods)
        elif model_type == "MLP-9":
            # shape-inconsistent in the reference too (model.py:71-78): the
            # second Linear expects input_dim features but receives 8
            self.layers = torch.nn.Sequential(
                torch.nn.Linear(input_dim, 8), torch.nn.ReLU(),
                torch.nn.Linear(input_dim, 16), torch.nn.ReLU(),
                torch.nn.Linear(16, output_dim))
        self.n_output_neurons = output_dim

    def forward(self, x: torch.FloatTensor) -> torch.FloatTensor:
        return self.layers(x)


def data_X_to_torch(data) -> torch.FloatTensor:
    """Creates torch training data (model.py:86-89)."""
    return torch.from_numpy(np.array(data).astype(np.float32))


def data_to_torch(data, labels) -> Tuple[torch.FloatTensor, torch.LongTensor]:
    data_X = data_X_to_torch(data)
    data_y = torch.as_tensor(torch.from_numpy(labels), dtype=torch.long)
    return data_X, data_y


def get_device() -> torch.device:
    """model.py:99-111 (cuda:0 there): the process's current device, which is
    cuda:0 in one process and the rank's own GPU under a launcher."""
    use_cuda = torch.cuda.is_available()
    device = torch.device("cuda", torch.cuda.current_device()) if use_cuda else torch.device("cpu")
    torch.backends.cudnn.benchmark = True
    return device


class NeuralNetwork(Logger):
    """The router (model.py:114-229); inference runs on K1 (lmi_router)."""

    # class-level defaults: an instance unpickled from the reference's own
    # pickle (li.index_io.load_index) carries only the reference's attributes
    _router = None
    _router_version = None

    def __init__(self, input_dim, output_dim, loss=torch.nn.CrossEntropyLoss, lr=0.1,
                 model_type="MLP", class_weight=None):
        self.device = get_device()
        self.model = Model(input_dim, output_dim, model_type=model_type).to(self.device)
        if class_weight is not None:
            self.loss = loss(weight=class_weight.to(self.device))
        else:
            self.loss = loss()
        self.optimizer = torch.optim.Adam(self.model.parameters(), lr=lr)
        self._router = None
        self._router_version = None

    def __getstate__(self):
        """Pickle what the reference pickles: the device router (ctypes
        descriptors over HBM) is rebuilt from the weights after loading."""
        st = dict(self.__dict__)
        st.pop("_router", None)
        st.pop("_router_version", None)
        return st

    # ---- training (index build; unchanged semantics, torch) ----------------
    def train(self, data_X, data_y, epochs=500, logger=None):
        step = epochs // 10
        losses = []
        if logger:
            logger.info(f"Epochs: {epochs}, step: {step}")
        for ep in range(epochs):
            pred_y = self.model(data_X.to(self.device))
            curr_loss = self.loss(pred_y, data_y.to(self.device))
            if ep % step == 0 and ep != 0 and logger:
                logger.info(f"Epoch {ep} | Loss {curr_loss.item()}")
            losses.append(curr_loss.item())
            self.model.zero_grad()
            curr_loss.backward()
            self.optimizer.step()
        return losses

    def train_batch(self, dataset, epochs=5, logger=None):
        """model.py:174-199, including its behaviour of stepping once per
        epoch on the last minibatch's loss."""
        step = max(epochs // 10, 1)
        losses = []
        if logger:
            logger.info(f"Epochs: {epochs}, step: {step}")
        for ep in range(epochs):
            for data_X, data_y in iter(dataset):
                pred_y = self.model(data_X.to(self.device))
                curr_loss = self.loss(pred_y, data_y.to(self.device))
            if ep % step == 0 and ep != 0 and logger:
                logger.info(f"Epoch {ep} | Loss {curr_loss.item():.5f}")
            losses.append(curr_loss.item())
            self.model.zero_grad()
            curr_loss.backward()
            self.optimizer.step()
        return losses

    # ---- inference on the GPU --------------------------------------------------
    def router(self):
        """DeviceRouter over the current weights (rebuilt after training)."""
        from .index import DeviceRouter
        version = tuple(p._version for p in self.model.parameters())
        if self._router is None or self._router_version != version:
            self._router = DeviceRouter.from_module(self.model, device=self.device)
            self._router_version = version
        return self._router

    def predict(self, data_X: torch.FloatTensor):
        """argmax of the logits (model.py:201-212) -> int64 ndarray."""
        self.model.eval()
        out = self.router().argmax(data_X.to(self.device))
        return out.cpu().numpy().astype(np.int64)

    def predict_proba(self, data_X: torch.FloatTensor):
        """(probs, classes) over all classes, descending (model.py:214-229).

        A 1-D input raises IndexError as the reference does: it takes the
        softmax over dim 0 and then `prob.topk(prob.shape[1])` (model.py:222-227)
        indexes a shape of length 1."""
        self.model.eval()
        x = data_X.to(self.device)
        if x.dim() == 1:
            raise IndexError("tuple index out of range (predict_proba of a 1-D input, "
                             "reference model.py:227)")
        r = self.router()
        classes, probs = r.topr(x, r.n_classes, with_probs=True)
        return probs.cpu().numpy(), classes.cpu().numpy().astype(np.int64)


class LIDataset(torch.utils.data.Dataset):
    def __init__(self, dataset_x, dataset_y):
        self.dataset_x, self.dataset_y = data_to_torch(dataset_x, dataset_y)

    def __len__(self):
        return self.dataset_x.shape[0]

    def __getitem__(self, idx):
        return self.dataset_x[idx - 1], self.dataset_y[idx - 1]
