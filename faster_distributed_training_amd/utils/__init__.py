from .env import (  # noqa: F401
    default_device, env_int, global_rank, has_gpu, is_rank0, local_rank, print0,
    seed_everything, world_size,
)
