"""paddle.distributed.launch — ``python -m paddle_ray_amd.distributed.launch --gpus 0,1 train.py``.

Parity: python/paddle/distributed/launch/main.py. One process per GPU on one
node, env: RANK/LOCAL_RANK/WORLD_SIZE/MASTER_ADDR/MASTER_PORT plus the paddle
names (PADDLE_TRAINER_ID, PADDLE_TRAINERS_NUM, FLAGS_selected_gpus). A failed
rank terminates its siblings (failure detection) and the launcher exits with
the first non-zero code.
"""
from .main import launch  # noqa
