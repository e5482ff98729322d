"""faster_distributed_training_amd — an MI355X-native fast-training engine.

Same capabilities as SuperbTUM/Faster-Distributed-Training (ResNet/CIFAR-10 and
Transformer/AG-News training with mixup, meta-mixup, online natural-gradient descent,
MADGRAD, mixed precision, DDP/FSDP, checkpoint/resume), re-designed for AMD Instinct
MI355X (gfx950 / CDNA4):

* hot ops are hand-written HIP kernels (``csrc/kernels/*.hip``) compiled into the
  in-tree extension ``_fdt_native`` (see ``ops/_native.py``);
* parameters, gradients and optimizer state live in flat HBM buffers
  (``utils/flat.py``) so optimizers, gradient clipping and gradient all-reduce are
  single launches / single collectives;
* communication is RCCL over xGMI through ``torch.distributed`` (backend ``nccl``),
  bucketed and overlapped with backward by our own reducer (``parallel/ddp.py``).
"""

__version__ = "0.1.0"

from . import utils  # noqa: F401
