"""CIFAR-10 data: dataset files, device-resident batches, GPU augmentation.

Reference: ``CIFAR10`` / ``VisionDataset`` (``resnet50_test.py:62-292``: pickled batches
kept as uint8 NHWC in RAM, per-sample float conversion), the scripted augmentation
(``:301-318``: RandomCrop(32, pad 4), RandomHorizontalFlip, Normalize) run per sample in
CPU workers, ``DataLoaderX`` + ``DistributedSampler`` (``:321-352``).

MI355X design: the whole uint8 training set (50000 x 32 x 32 x 3 = 153 MB) is uploaded
ONCE to HBM; a batch is a slice of a per-epoch permutation (DistributedSampler
semantics: identical seeded permutation on every rank, rank-strided shard,
``set_epoch``, ``drop_last``); one HIP kernel (``csrc/kernels/augment.hip``) gathers,
crops, flips, normalises and writes channels-last bf16 directly in the layout the conv
engine consumes.  No worker processes, no per-sample Python.  ``resident=False`` (image
sets larger than wanted in HBM) keeps the images on the host: each batch is gathered in
numpy and staged through the pinned ring + copy stream of ``prefetch.py`` one batch
ahead (the reference's pin_memory + non_blocking path), then augmented by the same
kernel.  The CPU path (tests, CPU training) implements the same transform with torch ops.

Fixed vs the reference: the transform order is deterministic crop -> flip -> normalise
(the reference permutes it randomly once per run, survey Q13); the sampler epoch is
advanced (Q10).
"""
from __future__ import annotations

import io
import os
import pickle

import numpy as np
import torch

from ..ops import _native

CIFAR_MEAN = (0.4914, 0.4822, 0.4465)
CIFAR_STD = (0.2023, 0.1994, 0.2010)
CLASSES = ('plane', 'car', 'bird', 'cat', 'deer', 'dog', 'frog', 'horse', 'ship', 'truck')

TRAIN_LIST = [("data_batch_1", "c99cafc152244af753f735de768cd75f"),
              ("data_batch_2", "d4bba439e000b95fd0a9bffe97cbabec"),
              ("data_batch_3", "54ebc095f3ab1f0389bbae665268c751"),
              ("data_batch_4", "634d18415352ddfa80567beed471001a"),
              ("data_batch_5", "482c414d41f54cd18b22e5b47cb7c3cb")]
TEST_LIST = [("test_batch", "40351d587109b95175f43aff81a1287e")]
BASE_FOLDER = "cifar-10-batches-py"
URL = "https://www.cs.toronto.edu/~kriz/cifar-10-python.tar.gz"
FILENAME = "cifar-10-python.tar.gz"
TGZ_MD5 = "c58f30108f718f92721af3b95e74349a"


def get_classes():
    return CLASSES


class _NumpyOnlyUnpickler(pickle.Unpickler):
    """The CIFAR python batches are pickles of dicts of numpy arrays.  Only the numpy
    array reconstruction machinery is allowed to load — anything else is refused."""
    ALLOWED = {("numpy.core.multiarray", "_reconstruct"), ("numpy", "ndarray"), ("numpy", "dtype"),
               ("numpy._core.multiarray", "_reconstruct"), ("numpy.core.multiarray", "scalar"),
               ("numpy._core.multiarray", "scalar"), ("_codecs", "encode")}

    def find_class(self, module, name):
        if (module, name) in self.ALLOWED:
            return super().find_class(module, name)
        raise pickle.UnpicklingError(f"refusing to load {module}.{name} from a CIFAR batch file")


def _load_batch(path):
    with open(path, "rb") as f:
        entry = _NumpyOnlyUnpickler(io.BytesIO(f.read()), encoding="latin1").load()
    data = np.asarray(entry["data"], dtype=np.uint8).reshape(-1, 3, 32, 32).transpose(0, 2, 3, 1)
    labels = entry["labels"] if "labels" in entry else entry["fine_labels"]
    return np.ascontiguousarray(data), np.asarray(labels, dtype=np.int64)


def _load_bin(path):
    raw = np.fromfile(path, dtype=np.uint8).reshape(-1, 3073)
    labels = raw[:, 0].astype(np.int64)
    data = raw[:, 1:].reshape(-1, 3, 32, 32).transpose(0, 2, 3, 1)
    return np.ascontiguousarray(data), labels


class CIFAR10:
    """Dataset holding uint8 NHWC images + int64 labels (D1).  Reads the python-pickle
    batches (``cifar-10-batches-py``, numpy-only unpickler) or the binary batches
    (``cifar-10-batches-bin``).  ``__getitem__`` returns (float CHW tensor, label) with
    the optional transform, for API parity with the reference class."""

    def __init__(self, root="./data", train=True, transform=None, target_transform=None, download=False):
        self.root = root
        self.train = train
        self.transform = transform
        self.target_transform = target_transform
        if download:
            self.download()
        self.data, self.targets = self._load()

    def _load(self):
        pyd = os.path.join(self.root, BASE_FOLDER)
        bind = os.path.join(self.root, "cifar-10-batches-bin")
        if os.path.isdir(pyd):
            names = [n for n, _ in (TRAIN_LIST if self.train else TEST_LIST)]
            parts = [_load_batch(os.path.join(pyd, n)) for n in names]
        elif os.path.isdir(bind):
            names = [f"data_batch_{i}.bin" for i in range(1, 6)] if self.train else ["test_batch.bin"]
            parts = [_load_bin(os.path.join(bind, n)) for n in names]
        else:
            raise RuntimeError(f"CIFAR-10 not found under {self.root} (use download=True or synthetic data)")
        return np.concatenate([p[0] for p in parts]), np.concatenate([p[1] for p in parts])

    def _check_integrity(self):
        from .download import check_integrity
        pyd = os.path.join(self.root, BASE_FOLDER)
        return all(check_integrity(os.path.join(pyd, n), md5) for n, md5 in TRAIN_LIST + TEST_LIST)

    def download(self):
        from .download import download_and_extract_archive
        if os.path.isdir(os.path.join(self.root, BASE_FOLDER)) and self._check_integrity():
            return
        download_and_extract_archive(URL, self.root, filename=FILENAME, md5=TGZ_MD5)

    def __len__(self):
        return len(self.data)

    def __getitem__(self, i):
        img = torch.from_numpy(self.data[i]).permute(2, 0, 1).float() / 255.0
        if self.transform is not None:
            img = self.transform(img)
        t = int(self.targets[i])
        if self.target_transform is not None:
            t = self.target_transform(t)
        return img, t


def synthetic_cifar(n=50000, num_classes=10, seed=0, hw=32):
    """CIFAR-shaped synthetic uint8 data (benchmarks: no network for the dataset)."""
    g = torch.Generator().manual_seed(seed)
    data = torch.randint(0, 256, (n, hw, hw, 3), generator=g, dtype=torch.uint8).numpy()
    targets = torch.randint(0, num_classes, (n,), generator=g).numpy()
    return data, targets


# ------------------------------------------------------------------ CPU transforms
TRANSFORMS = ("crop", "flip", "normalize")


def augment_order(seed: int | None = None, faithful: bool = False):
    """Order of the train transforms.  The reference draws a random permutation of
    (RandomCrop, RandomHorizontalFlip, Normalize) once per run with
    ``np.random.choice(range(3), 3, replace=False)`` (resnet50_test.py:304-309, survey Q13);
    ``faithful`` reproduces that draw from a seeded generator, the default is the fixed
    torchvision order crop -> flip -> normalise."""
    if not faithful:
        return TRANSFORMS
    perm = np.random.RandomState(seed).choice(range(3), 3, replace=False)
    return tuple(TRANSFORMS[i] for i in perm)


def pad_normalized(order) -> bool:
    """True when normalisation precedes the zero-padded crop (padding is then 0 in
    normalised space); flip commutes with both in distribution (csrc/kernels/augment.hip)."""
    return order.index("normalize") < order.index("crop")


def augment_cpu(imgs_u8: torch.Tensor, gen: torch.Generator | None = None, pad=4, flip=True, train=True,
                out_dtype=torch.float32, channels_last=False, order=TRANSFORMS):
    """Reference-semantics batch transform on CPU: uint8 NHWC -> normalised NCHW float."""
    x = imgs_u8.permute(0, 3, 1, 2).float() / 255.0
    B, C, H, W = x.shape
    mean = torch.tensor(CIFAR_MEAN).view(1, 3, 1, 1)
    std = torch.tensor(CIFAR_STD).view(1, 3, 1, 1)
    norm_first = train and pad > 0 and pad_normalized(order)
    if norm_first:
        x = (x - mean) / std
    if train and pad > 0:
        xp = torch.nn.functional.pad(x, (pad, pad, pad, pad))
        dy = torch.randint(0, 2 * pad + 1, (B,), generator=gen)
        dx = torch.randint(0, 2 * pad + 1, (B,), generator=gen)
        rows = (dy.view(B, 1) + torch.arange(H).view(1, H))
        cols = (dx.view(B, 1) + torch.arange(W).view(1, W))
        x = xp[torch.arange(B).view(B, 1, 1, 1), torch.arange(C).view(1, C, 1, 1), rows.view(B, 1, H, 1),
               cols.view(B, 1, 1, W)]
    if train and flip:
        f = torch.rand(B, generator=gen) < 0.5
        x = torch.where(f.view(B, 1, 1, 1), x.flip(3), x)
    if not norm_first:
        x = (x - mean) / std
    x = x.to(out_dtype)
    if channels_last:
        x = x.contiguous(memory_format=torch.channels_last)
    return x


# ------------------------------------------------------------------ loader
class DeviceCIFARLoader:
    """Device-resident CIFAR batches with GPU augmentation (D2/D4/D5/D7 in one).

    Iterating yields ``(images, labels)``; on GPU images are channels-last bf16 NCHW
    views (the conv engine consumes them with zero copies).  ``set_epoch`` reseeds the
    shared permutation (DistributedSampler semantics)."""

    def __init__(self, data_u8, targets, batch_size, device, train=True, rank=0, world_size=1, seed=0,
                 drop_last=True, shuffle=True, out_dtype=torch.bfloat16, pad=4, flip=True, augment=True,
                 order=TRANSFORMS, resident=True):
        self.device = torch.device(device)
        self.train = train
        self.bs = batch_size
        self.rank, self.world = rank, world_size
        self.seed = seed
        self.drop_last = drop_last
        self.shuffle = shuffle
        self.out_dtype = out_dtype
        self.pad, self.flip, self.augment = pad, flip, augment
        self.order = tuple(order)
        self.n = len(targets)
        self._gpu = self.device.type == "cuda" and _native.enabled()
        self.resident = resident or not self._gpu
        self.stager = None
        if self.resident:
            self.images = torch.as_tensor(np.ascontiguousarray(data_u8)).to(self.device)
            self.labels = torch.as_tensor(np.asarray(targets)).to(torch.int32).to(self.device)
        else:
            from .prefetch import PinnedStager
            self.host_images = np.ascontiguousarray(data_u8)
            self.host_labels = np.asarray(targets).astype(np.int32)
            per = batch_size * int(np.prod(self.host_images.shape[1:])) + 4 * batch_size + 512
            self.stager = PinnedStager(self.device, per, 3)
            self._iota = torch.arange(batch_size, dtype=torch.int32, device=self.device)
        self.epoch = 0
        # per-rank stream of crop / flip draws (the kernel hashes (seed, step, sample))
        self.rng = torch.tensor([seed + 7919 * rank, 0], dtype=torch.int64, device=self.device)
        self._cpu_gen = torch.Generator().manual_seed(seed + 7919 * rank)

    def set_epoch(self, epoch: int):
        self.epoch = epoch

    def _indices(self):
        if self.shuffle:
            g = torch.Generator().manual_seed(self.seed + self.epoch)
            perm = torch.randperm(self.n, generator=g)
        else:
            perm = torch.arange(self.n)
        per_rank = self.n // self.world if self.drop_last else -(-self.n // self.world)
        if not self.drop_last:
            pad = per_rank * self.world - self.n
            if pad:
                perm = torch.cat([perm, perm[:pad]])
        shard = perm[self.rank:per_rank * self.world:self.world]
        return shard

    def __len__(self):
        per_rank = self.n // self.world if self.drop_last else -(-self.n // self.world)
        return per_rank // self.bs if self.drop_last else -(-per_rank // self.bs)

    def batch(self, idx: torch.Tensor, images=None, labels=None):
        """Augment one batch given sample indices (device int32) into ``images`` /
        ``labels`` (default: the resident set)."""
        B = idx.numel()
        if self._gpu:
            nat = _native.native()
            images = self.images if images is None else images
            labels = self.labels if labels is None else labels
            # NHWC with channels zero-padded to 8: the conv engine's stem operand layout
            cp = 8
            out = torch.empty(B, 32, 32, cp, device=self.device, dtype=self.out_dtype)
            lab = torch.empty(B, device=self.device, dtype=torch.int32)
            train = self.train and self.augment
            nat.augment(images.data_ptr(), idx.data_ptr(), labels.data_ptr(), lab.data_ptr(),
                        out.data_ptr(), B, 32, 32, 3, cp, self.pad if train else 0, int(train and self.flip),
                        self.rng.data_ptr(), *CIFAR_MEAN, *CIFAR_STD, 0, int(pad_normalized(self.order)),
                        1 if self.out_dtype == torch.bfloat16 else 0, _native.stream_ptr())
            nat.rng_advance(self.rng.data_ptr(), _native.stream_ptr())
            return out[..., :3].permute(0, 3, 1, 2), lab.long()
        imgs = self.images[idx.long()].cpu()
        x = augment_cpu(imgs, self._cpu_gen, pad=self.pad, flip=self.flip, train=self.train and self.augment,
                        out_dtype=torch.float32, order=self.order)
        return x.to(self.device), self.labels[idx.long()].long()

    def _host(self, shard, b):
        sel = shard[b * self.bs:(b + 1) * self.bs]
        return [np.take(self.host_images, sel, axis=0), self.host_labels[sel]], None

    def _device(self, arrs, _meta):
        imgs, labs = arrs
        return self.batch(self._iota[:imgs.shape[0]], images=imgs, labels=labs)

    def __iter__(self):
        shard = self._indices()
        nb = len(self)
        if not self.resident:
            from .prefetch import StagedIterator
            sh = shard.numpy()
            yield from StagedIterator(self.stager, nb, lambda b: self._host(sh, b), self._device)
            return
        # one index upload per epoch, from pinned memory on the compute stream (no host sync)
        idx_cpu = shard.to(torch.int32)
        if self.device.type == "cuda":
            idx_cpu = idx_cpu.pin_memory()
        idx_all = idx_cpu.to(self.device, non_blocking=True)
        for b in range(nb):
            idx = idx_all[b * self.bs:(b + 1) * self.bs]
            if idx.numel() == 0:
                break
            yield self.batch(idx)
