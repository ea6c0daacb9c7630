"""paddle.geometric.message_passing import path (reference python/paddle/geometric/
message_passing/send_recv.py)."""
from .. import send_u_recv, send_ue_recv, send_uv  # noqa: F401

__all__ = []
