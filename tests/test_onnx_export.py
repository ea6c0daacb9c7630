"""paddle.onnx.export: self-contained ONNX writer (aten ops recorded on CPU -> ONNX nodes, constants
folded into initializers) checked by evaluating the exported file with the NumPy runtime
(paddle.onnx.run) against the layer itself, and by parsing the bytes with google.protobuf
messages built from the onnx.proto field numbers. Parity: python/paddle/onnx/export.py (which
delegates to paddle2onnx; no reference fixture exists, so the format check is against onnx.proto)."""
import numpy as np
import pytest
import torch

import paddle_ray_amd as paddle
from paddle_ray_amd import nn, onnx as O
from paddle_ray_amd.static import InputSpec


def _check(layer, shape, tmp_path, tol=1e-4, dtype='float32', gen=None):
    layer.eval()
    spec = [InputSpec(shape, dtype)]
    fn = O.export(layer, str(tmp_path / 'm'), spec, opset_version=13)
    x = gen() if gen else np.random.RandomState(0).randn(*shape).astype(np.float32)
    y, = O.run(fn, [x])
    ref = layer(paddle.to_tensor(x)).numpy()
    assert y.shape == ref.shape
    np.testing.assert_allclose(y, ref, rtol=tol, atol=tol)
    return fn


def test_lenet(tmp_path):
    from paddle_ray_amd.vision.models import LeNet
    paddle.seed(0)
    _check(LeNet(), [2, 1, 28, 28], tmp_path)


def test_resnet18_bn_pool(tmp_path):
    from paddle_ray_amd.vision.models import resnet18
    paddle.seed(1)
    m = resnet18(num_classes=10)
    for p in m.buffers():          # non-trivial BN running statistics
        p._t.uniform_(0.5, 1.5)
    _check(m, [1, 3, 32, 32], tmp_path, tol=2e-3)


class _Block(nn.Layer):
    def __init__(self):
        super().__init__()
        self.emb = nn.Embedding(50, 32)
        self.ln = nn.LayerNorm(32)
        self.fc1 = nn.Linear(32, 64)
        self.fc2 = nn.Linear(64, 5)

    def forward(self, ids):
        h = self.ln(self.emb(ids))
        h = nn.functional.gelu(self.fc1(h))
        return nn.functional.softmax(self.fc2(h).mean(axis=1), axis=-1)


def test_embedding_layernorm_gelu_softmax(tmp_path):
    paddle.seed(2)
    _check(_Block(), [3, 7], tmp_path, dtype='int64',
           gen=lambda: np.random.RandomState(3).randint(0, 50, (3, 7)).astype(np.int64))


class _Up(nn.Layer):
    """Decoder-style upsampling: transposed convolutions with stride, padding, output padding,
    dilation and groups (ONNX ConvTranspose)."""

    def __init__(self):
        super().__init__()
        self.a = nn.Conv2DTranspose(4, 6, 3, stride=2, padding=1, output_padding=1)
        self.b = nn.Conv2DTranspose(6, 4, 4, stride=2, padding=1, groups=2)
        self.c = nn.Conv2DTranspose(4, 3, 3, stride=1, padding=2, dilation=2, bias_attr=False)

    def forward(self, x):
        return self.c(nn.functional.relu(self.b(nn.functional.relu(self.a(x)))))


def test_conv_transpose(tmp_path):
    paddle.seed(4)
    _check(_Up(), [2, 4, 5, 7], tmp_path)


def test_unsupported_op_is_named(tmp_path):
    class Odd(nn.Layer):
        def forward(self, x):
            return paddle.Tensor(torch.fft.fft(x._t).real)
    with pytest.raises(NotImplementedError, match='aten'):
        O.export(Odd(), str(tmp_path / 'odd'), [InputSpec([4, 8], 'float32')])


def test_bytes_parse_with_google_protobuf(tmp_path):
    from google.protobuf import descriptor_pb2, descriptor_pool, message_factory
    from paddle_ray_amd.vision.models import LeNet
    fd = descriptor_pb2.FileDescriptorProto(name='onnx_subset.proto', package='onnx', syntax='proto2')
    F = descriptor_pb2.FieldDescriptorProto

    def msg(name, fields):
        m = fd.message_type.add(name=name)
        for num, fname, typ, label, tname in fields:
            f = m.field.add(name=fname, number=num, type=typ, label=label)
            if tname:
                f.type_name = '.onnx.' + tname
    O_, R_ = F.LABEL_OPTIONAL, F.LABEL_REPEATED
    msg('OperatorSetIdProto', [(1, 'domain', F.TYPE_STRING, O_, None), (2, 'version', F.TYPE_INT64, O_, None)])
    msg('Dimension', [(1, 'dim_value', F.TYPE_INT64, O_, None), (2, 'dim_param', F.TYPE_STRING, O_, None)])
    msg('TensorShapeProto', [(1, 'dim', F.TYPE_MESSAGE, R_, 'Dimension')])
    msg('TypeTensor', [(1, 'elem_type', F.TYPE_INT32, O_, None), (2, 'shape', F.TYPE_MESSAGE, O_, 'TensorShapeProto')])
    msg('TypeProto', [(1, 'tensor_type', F.TYPE_MESSAGE, O_, 'TypeTensor')])
    msg('ValueInfoProto', [(1, 'name', F.TYPE_STRING, O_, None), (2, 'type', F.TYPE_MESSAGE, O_, 'TypeProto')])
    msg('TensorProto', [(1, 'dims', F.TYPE_INT64, R_, None), (2, 'data_type', F.TYPE_INT32, O_, None),
                        (8, 'name', F.TYPE_STRING, O_, None), (9, 'raw_data', F.TYPE_BYTES, O_, None)])
    msg('AttributeProto', [(1, 'name', F.TYPE_STRING, O_, None), (2, 'f', F.TYPE_FLOAT, O_, None),
                           (3, 'i', F.TYPE_INT64, O_, None), (4, 's', F.TYPE_BYTES, O_, None),
                           (7, 'floats', F.TYPE_FLOAT, R_, None), (8, 'ints', F.TYPE_INT64, R_, None),
                           (20, 'type', F.TYPE_INT32, O_, None)])
    msg('NodeProto', [(1, 'input', F.TYPE_STRING, R_, None), (2, 'output', F.TYPE_STRING, R_, None),
                      (3, 'name', F.TYPE_STRING, O_, None), (4, 'op_type', F.TYPE_STRING, O_, None),
                      (5, 'attribute', F.TYPE_MESSAGE, R_, 'AttributeProto')])
    msg('GraphProto', [(1, 'node', F.TYPE_MESSAGE, R_, 'NodeProto'), (2, 'name', F.TYPE_STRING, O_, None),
                       (5, 'initializer', F.TYPE_MESSAGE, R_, 'TensorProto'),
                       (11, 'input', F.TYPE_MESSAGE, R_, 'ValueInfoProto'),
                       (12, 'output', F.TYPE_MESSAGE, R_, 'ValueInfoProto')])
    msg('ModelProto', [(1, 'ir_version', F.TYPE_INT64, O_, None), (2, 'producer_name', F.TYPE_STRING, O_, None),
                       (3, 'producer_version', F.TYPE_STRING, O_, None), (7, 'graph', F.TYPE_MESSAGE, O_, 'GraphProto'),
                       (8, 'opset_import', F.TYPE_MESSAGE, R_, 'OperatorSetIdProto')])
    pool = descriptor_pool.DescriptorPool()
    pool.Add(fd)
    Model = message_factory.GetMessageClass(pool.FindMessageTypeByName('onnx.ModelProto'))
    paddle.seed(0)
    fn = O.export(LeNet(), str(tmp_path / 'lenet'), [InputSpec([1, 1, 28, 28], 'float32')], opset_version=13)
    m = Model()
    m.ParseFromString(open(fn, 'rb').read())
    assert m.opset_import[0].version == 13 and m.producer_name == 'paddle_ray_amd'
    ops = [n.op_type for n in m.graph.node]
    assert 'Conv' in ops and 'MaxPool' in ops and 'Gemm' in ops
    assert [d.dim_value for d in m.graph.input[0].type.tensor_type.shape.dim] == [1, 1, 28, 28]
    w = [t for t in m.graph.initializer if len(t.dims) == 4][0]
    assert w.data_type == 1 and len(w.raw_data) == 4 * int(np.prod(list(w.dims)))
    # and our decoder reads what protobuf re-serialises
    assert O._dec('ModelProto', m.SerializeToString())['graph']['node'][0]['op_type'] == ops[0]


def test_gpt_and_bert_export(tmp_path):
    """Attention models (causal GPT with the tied LM head, BERT encoder + pooler): the flash
    attention reference path (masked scores, logsumexp, softmax) exports and matches."""
    from paddle_ray_amd.models import gpt_config, GPTForPretraining, BertModel, bert_config
    paddle.seed(0)
    ids = np.random.RandomState(0).randint(0, 1000, (2, 16)).astype(np.int64)
    m = GPTForPretraining(gpt_config('gpt3-tiny', hidden_dropout=0.0, attention_dropout=0.0))
    m.eval()
    fn = O.export(m, str(tmp_path / 'gpt'), [InputSpec([2, 16], 'int64')], opset_version=13)
    y, = O.run(fn, [ids])
    np.testing.assert_allclose(y, m(paddle.to_tensor(ids)).numpy(), rtol=1e-4, atol=1e-4)
    cfg = bert_config('bert-base-uncased', num_hidden_layers=1, hidden_dropout_prob=0.0,
                      attention_probs_dropout_prob=0.0)
    bm = BertModel(cfg)
    bm.eval()
    fn = O.export(bm, str(tmp_path / 'bert'), [InputSpec([2, 16], 'int64')], opset_version=13)
    seq, pooled = O.run(fn, [ids])
    rs, rp = bm(paddle.to_tensor(ids))
    np.testing.assert_allclose(seq, rs.numpy(), rtol=1e-4, atol=1e-4)
    np.testing.assert_allclose(pooled, rp.numpy(), rtol=1e-4, atol=1e-4)


@pytest.mark.parametrize('name', ['mobilenet_v2', 'mobilenet_v3_small', 'resnet50_nhwc'])
def test_vision_zoo_export(name, tmp_path):
    """Depthwise convs, hardswish / SE blocks, channels-last ResNet (permutes, in-place restrides)."""
    from paddle_ray_amd.vision import models as M
    paddle.seed(0)
    if name == 'resnet50_nhwc':
        m, shape = M.resnet50(num_classes=10, data_format='NHWC'), [1, 32, 32, 3]
    else:
        m, shape = getattr(M, name)(num_classes=10), [1, 3, 32, 32]
    _check(m, shape, tmp_path, tol=2e-3)
