"""ProgramDesc protobuf .pdmodel (static/program_desc.py) checked against an independent
protobuf implementation: google.protobuf messages built at run time from a descriptor that
transcribes framework.proto (reference: paddle/fluid/framework/framework.proto:23-246; the
field numbers / types below are that file's)."""
import numpy as np
import pytest

import paddle_ray_amd as paddle
from paddle_ray_amd import static
from paddle_ray_amd.static import program_desc as PD

pb = pytest.importorskip('google.protobuf')
from google.protobuf import descriptor_pb2, descriptor_pool, message_factory  # noqa: E402

F = descriptor_pb2.FieldDescriptorProto


def _msg(fp, name, fields, nested=()):
    m = fp.message_type.add() if not isinstance(fp, descriptor_pb2.DescriptorProto) \
        else fp.nested_type.add()
    m.name = name
    for num, fname, ftype, label, tname in fields:
        f = m.field.add()
        f.name, f.number, f.type, f.label = fname, num, ftype, label
        if tname:
            f.type_name = tname
    for n in nested:
        n(m)
    return m


def _framework_proto():
    fp = descriptor_pb2.FileDescriptorProto()
    fp.name, fp.package, fp.syntax = 'fw_test.proto', 'fwt', 'proto2'
    O, R, Q = F.LABEL_OPTIONAL, F.LABEL_REPEATED, F.LABEL_REQUIRED
    _msg(fp, 'Version', [(1, 'version', F.TYPE_INT64, O, None)])

    def attr(m):
        _msg(m, 'Attr', [(1, 'name', F.TYPE_STRING, Q, None), (2, 'type', F.TYPE_INT32, Q, None),
                         (3, 'i', F.TYPE_INT32, O, None), (4, 'f', F.TYPE_FLOAT, O, None),
                         (5, 's', F.TYPE_STRING, O, None), (6, 'ints', F.TYPE_INT32, R, None),
                         (10, 'b', F.TYPE_BOOL, O, None), (12, 'block_idx', F.TYPE_INT32, O, None),
                         (13, 'l', F.TYPE_INT64, O, None), (15, 'longs', F.TYPE_INT64, R, None),
                         (16, 'float64s', F.TYPE_DOUBLE, R, None),
                         (19, 'float64', F.TYPE_DOUBLE, O, None)])

    def var(m):
        _msg(m, 'Var', [(1, 'parameter', F.TYPE_STRING, Q, None),
                        (2, 'arguments', F.TYPE_STRING, R, None)])
    _msg(fp, 'OpDesc', [(3, 'type', F.TYPE_STRING, Q, None),
                        (1, 'inputs', F.TYPE_MESSAGE, R, '.fwt.OpDesc.Var'),
                        (2, 'outputs', F.TYPE_MESSAGE, R, '.fwt.OpDesc.Var'),
                        (4, 'attrs', F.TYPE_MESSAGE, R, '.fwt.OpDesc.Attr'),
                        (5, 'is_target', F.TYPE_BOOL, O, None)], nested=(attr, var))

    def tdesc(m):
        _msg(m, 'TensorDesc', [(1, 'data_type', F.TYPE_INT32, Q, None),
                               (2, 'dims', F.TYPE_INT64, R, None)])

    def ldesc(m):
        _msg(m, 'LoDTensorDesc', [(1, 'tensor', F.TYPE_MESSAGE, Q, '.fwt.VarType.TensorDesc'),
                                  (2, 'lod_level', F.TYPE_INT32, O, None)])
    _msg(fp, 'VarType', [(1, 'type', F.TYPE_INT32, Q, None),
                         (3, 'lod_tensor', F.TYPE_MESSAGE, O, '.fwt.VarType.LoDTensorDesc')],
         nested=(tdesc, ldesc))
    _msg(fp, 'VarDesc', [(1, 'name', F.TYPE_STRING, Q, None),
                         (2, 'type', F.TYPE_MESSAGE, Q, '.fwt.VarType'),
                         (3, 'persistable', F.TYPE_BOOL, O, None),
                         (4, 'need_check_feed', F.TYPE_BOOL, O, None),
                         (5, 'is_parameter', F.TYPE_BOOL, O, None),
                         (6, 'stop_gradient', F.TYPE_BOOL, O, None)])
    _msg(fp, 'BlockDesc', [(1, 'idx', F.TYPE_INT32, Q, None), (2, 'parent_idx', F.TYPE_INT32, Q, None),
                           (3, 'vars', F.TYPE_MESSAGE, R, '.fwt.VarDesc'),
                           (4, 'ops', F.TYPE_MESSAGE, R, '.fwt.OpDesc'),
                           (5, 'forward_block_idx', F.TYPE_INT32, O, None)])
    _msg(fp, 'ProgramDesc', [(1, 'blocks', F.TYPE_MESSAGE, R, '.fwt.BlockDesc'),
                             (4, 'version', F.TYPE_MESSAGE, O, '.fwt.Version')])
    pool = descriptor_pool.DescriptorPool()
    pool.Add(fp)
    desc = pool.FindMessageTypeByName('fwt.ProgramDesc')
    try:
        return message_factory.GetMessageClass(desc)
    except AttributeError:  # older protobuf
        return message_factory.MessageFactory(pool).GetPrototype(desc)


def test_codec_roundtrip_and_negative_varints():
    d = {'blocks': [{'idx': 0, 'parent_idx': -1, 'vars': [PD.var_desc('x', [-1, 4], 'bfloat16')],
                     'ops': [{'type': 't', 'attrs': [PD.scalar_attr('k', -3),
                                                     PD.scalar_attr('big', 2 ** 40),
                                                     PD.scalar_attr('fs', [0.5, 2]),
                                                     PD.scalar_attr('on', True)]}]}],
         'version': {'version': PD.PROGRAM_VERSION}}
    back = PD.decode('ProgramDesc', PD.encode('ProgramDesc', d))
    b = back['blocks'][0]
    assert b['parent_idx'] == -1
    assert PD.var_info(b['vars'][0]) == ('x', [-1, 4], 'bfloat16')
    vals = {a['name']: PD.attr_value(a) for a in b['ops'][0]['attrs']}
    assert vals == {'k': -3, 'big': 2 ** 40, 'fs': [0.5, 2.0], 'on': True}


def test_saved_pdmodel_parses_as_framework_proto(tmp_path):
    Program = _framework_proto()
    paddle.enable_static()
    try:
        main = static.Program()
        with static.program_guard(main):
            x = static.data('x', [None, 4], 'float32')
            h = paddle.nn.functional.relu(static.nn.fc(x, 3))
            y = paddle.nn.functional.softmax(h, axis=-1)
        exe = static.Executor()
        path = str(tmp_path / 'm')
        static.save_inference_model(path, [x], [y], exe, program=main)
        msg = Program()
        msg.ParseFromString(open(path + '.pdmodel', 'rb').read())
        assert msg.IsInitialized()  # every proto2 `required` field is present
        b0 = msg.blocks[0]
        assert b0.idx == 0 and b0.parent_idx == -1 and msg.version.version == PD.PROGRAM_VERSION
        types = [o.type for o in b0.ops]
        assert types[0] == 'feed' and types[-1] == 'fetch'
        assert any(t.endswith(':relu') for t in types) and any(t.endswith(':softmax') for t in types)
        sm = next(o for o in b0.ops if o.type.endswith(':softmax'))
        assert {a.name: a.i for a in sm.attrs if a.type == PD.ATTR['INT']}.get('axis') == -1
        vars_ = {v.name: v for v in b0.vars}
        xin = vars_[b0.ops[0].outputs[0].arguments[0]]
        assert list(xin.type.lod_tensor.tensor.dims) == [-1, 4] and xin.need_check_feed
        assert xin.type.lod_tensor.tensor.data_type == 5  # FP32
        params = [v for v in b0.vars if v.is_parameter]
        assert len(params) == 2 and all(v.persistable for v in params)
        prog, feeds, fetches = static.load_inference_model(path, exe)
        xv = np.random.RandomState(0).randn(3, 4).astype('float32')
        ref = exe.run(main, feed={'x': xv}, fetch_list=[y])[0]
        got = exe.run(prog, feed={feeds[0]: xv}, fetch_list=fetches)[0]
        np.testing.assert_allclose(got, ref, rtol=1e-6)
    finally:
        paddle.disable_static()
