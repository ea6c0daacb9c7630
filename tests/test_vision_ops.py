"""paddle.vision.ops (parity: test/legacy_test/test_roi_align_op.py, test_nms_op.py,
test_box_coder_op.py, test_prior_box_op.py, test_yolo_box_op.py, test_yolov3_loss_op.py,
test_deformable_conv_op.py, test_matrix_nms_op.py, test_distribute_fpn_proposals_op.py)."""
import io

import numpy as np
import pytest
import torch

import paddle_ray_amd as paddle
from paddle_ray_amd.vision import ops as V


def test_roi_align_linear_ramp_exact():
    # f(y, x) = x: every bilinear sample returns its x, so a bin average is its center x
    H = W = 16
    x = paddle.to_tensor(np.tile(np.arange(W, dtype=np.float32), (1, 2, H, 1)))
    boxes = paddle.to_tensor(np.array([[2.0, 3.0, 10.0, 11.0]], np.float32))
    out = V.roi_align(x, boxes, paddle.to_tensor([1]), output_size=4, sampling_ratio=2,
                      aligned=True).numpy()
    assert out.shape == (1, 2, 4, 4)
    centers = 2.0 - 0.5 + (np.arange(4) + 0.5) * 2.0
    np.testing.assert_allclose(out[0, 0, 0], centers, atol=1e-5)
    np.testing.assert_allclose(out[0, 1, 3], centers, atol=1e-5)


def test_roi_align_grad_and_batch_index():
    x = paddle.randn([2, 3, 8, 8])
    x.stop_gradient = False
    boxes = paddle.to_tensor(np.array([[0, 0, 4, 4], [1, 1, 7, 7], [2, 2, 6, 6]], np.float32))
    out = V.RoIAlign(2)(x, boxes, paddle.to_tensor([1, 2]))
    out.sum().backward()
    g = x.grad.numpy()
    assert out.shape == [3, 3, 2, 2] and np.abs(g[0]).sum() > 0 and np.abs(g[1]).sum() > 0


def test_roi_pool_max():
    x = np.zeros((1, 1, 8, 8), np.float32)
    x[0, 0, 1, 1], x[0, 0, 6, 6] = 5.0, 7.0
    out = V.roi_pool(paddle.to_tensor(x), paddle.to_tensor(np.array([[0, 0, 7, 7]], np.float32)),
                     paddle.to_tensor([1]), output_size=2).numpy()
    np.testing.assert_allclose(out[0, 0], [[5, 0], [0, 7]])


def test_psroi_pool_channels():
    x = np.zeros((1, 2 * 4, 4, 4), np.float32)
    for c in range(8):
        x[0, c] = c
    out = V.psroi_pool(paddle.to_tensor(x), paddle.to_tensor(np.array([[0, 0, 3, 3]],
                                                                      np.float32)),
                       paddle.to_tensor([1]), output_size=2).numpy()
    np.testing.assert_allclose(out[0].reshape(-1), np.arange(8, dtype=np.float32))


def test_nms():
    boxes = paddle.to_tensor(np.array([[0, 0, 10, 10], [1, 1, 11, 11], [20, 20, 30, 30],
                                       [21, 21, 31, 31]], np.float32))
    scores = paddle.to_tensor(np.array([0.9, 0.95, 0.5, 0.3], np.float32))
    assert V.nms(boxes, 0.5, scores).numpy().tolist() == [1, 2]
    assert V.nms(boxes, 0.5).numpy().tolist() == [0, 2]
    cats = paddle.to_tensor(np.array([0, 1, 0, 0]))
    assert sorted(V.nms(boxes, 0.5, scores, cats, [0, 1]).numpy().tolist()) == [0, 1, 2]
    assert V.nms(boxes, 0.5, scores, top_k=1).numpy().tolist() == [1]


def test_box_coder_roundtrip():
    rs = np.random.RandomState(0)
    prior = np.sort(rs.rand(5, 4).astype(np.float32).reshape(5, 2, 2), axis=1).reshape(5, 4)
    prior = prior[:, [0, 2, 1, 3]]
    target = prior + 0.01
    var = [0.1, 0.1, 0.2, 0.2]
    enc = V.box_coder(paddle.to_tensor(prior), var, paddle.to_tensor(target))
    assert enc.shape == [5, 5, 4]
    dec = V.box_coder(paddle.to_tensor(prior), var, enc, code_type='decode_center_size')
    np.testing.assert_allclose(dec.numpy()[np.arange(5), np.arange(5)], target, atol=1e-5)


def test_prior_box():
    feat = paddle.zeros([1, 8, 4, 4])
    img = paddle.zeros([1, 3, 32, 32])
    boxes, var = V.prior_box(feat, img, min_sizes=[8.0], max_sizes=[16.0],
                             aspect_ratios=[2.0], flip=True, clip=True)
    assert boxes.shape == [4, 4, 4, 4] and var.shape == [4, 4, 4, 4]
    b = boxes.numpy()[0, 0, 0]  # cell (0,0) center (4,4), square min size 8
    np.testing.assert_allclose(b, [0.0, 0.0, 8 / 32, 8 / 32], atol=1e-6)


def test_yolo_box_and_loss():
    paddle.seed(0)
    anchors = [10, 13, 16, 30, 33, 23]
    x = paddle.randn([2, 3 * (5 + 4), 4, 4])
    boxes, scores = V.yolo_box(x, paddle.to_tensor(np.array([[64, 64], [64, 64]])), anchors,
                               4, 0.01, 16)
    assert boxes.shape == [2, 48, 4] and scores.shape == [2, 48, 4]
    b = boxes.numpy()
    assert (b >= 0).all() and (b <= 63).all()
    gt = paddle.to_tensor(np.array([[[0.5, 0.5, 0.3, 0.4], [0.2, 0.3, 0.1, 0.1]]] * 2,
                                   np.float32))
    lab = paddle.to_tensor(np.array([[1, 2]] * 2))
    w = paddle.create_parameter([2, 27, 4, 4], 'float32')
    opt = paddle.optimizer.Adam(learning_rate=0.05, parameters=[w])
    losses = []
    for _ in range(20):
        loss = V.yolo_loss(w, gt, lab, anchors, [0, 1, 2], 4, 0.7, 16).sum()
        loss.backward()
        opt.step()
        opt.clear_grad()
        losses.append(float(loss))
    assert np.isfinite(losses).all() and losses[-1] < losses[0]


def test_deform_conv_zero_offset_is_conv():
    paddle.seed(1)
    x = paddle.randn([2, 4, 7, 7])
    layer = V.DeformConv2D(4, 6, 3, padding=1, groups=2, deformable_groups=2)
    off = paddle.zeros([2, 2 * 2 * 9, 7, 7])
    mask = paddle.ones([2, 2 * 9, 7, 7])
    ref = paddle.nn.functional.conv2d(x, layer.weight, layer.bias, padding=1, groups=2)
    np.testing.assert_allclose(layer(x, off, mask).numpy(), ref.numpy(), atol=1e-4)
    np.testing.assert_allclose(layer(x, off).numpy(), ref.numpy(), atol=1e-4)
    # integer shift of +1 in x equals sampling the right neighbour
    off2 = np.zeros((2, 36, 7, 7), np.float32)
    off2[:, 1::2] = 1.0
    xs = np.pad(x.numpy(), ((0, 0), (0, 0), (0, 0), (0, 1)))[..., 1:]
    ref2 = paddle.nn.functional.conv2d(paddle.to_tensor(xs), layer.weight, layer.bias,
                                       padding=1, groups=2)
    # (output column 0 differs: its shifted left tap reads x[0], the padded reference 0)
    np.testing.assert_allclose(layer(x, paddle.to_tensor(off2)).numpy()[..., 1:],
                               ref2.numpy()[..., 1:], atol=1e-4)


def test_matrix_nms():
    bboxes = paddle.to_tensor(np.array([[[0, 0, 1, 1], [0, 0, 1, 1.05], [2, 2, 3, 3]]],
                                       np.float32))
    scores = paddle.to_tensor(np.array([[[0.0, 0.0, 0.0], [0.9, 0.8, 0.7]]], np.float32))
    out, idx, num = V.matrix_nms(bboxes, scores, 0.1, 0.3, -1, -1, return_index=True)
    o = out.numpy()
    assert num.numpy().tolist() == [2] and o[0, 1] == pytest.approx(0.9)
    assert idx.numpy().reshape(-1).tolist() == [0, 2]


def test_distribute_fpn_and_proposals():
    rois = paddle.to_tensor(np.array([[0, 0, 10, 10], [0, 0, 200, 200], [0, 0, 60, 60],
                                      [0, 0, 500, 500]], np.float32))
    multi, restore, nums = V.distribute_fpn_proposals(rois, 2, 5, 4, 224,
                                                      rois_num=paddle.to_tensor([2, 2]))
    cat = np.concatenate([m.numpy() for m in multi])
    np.testing.assert_allclose(cat[restore.numpy().reshape(-1)], rois.numpy())
    assert sum(int(n.numpy().sum()) for n in nums) == 4
    paddle.seed(0)
    A, H, W = 3, 4, 4
    anchors = np.zeros((H, W, A, 4), np.float32)
    for i in range(H):
        for j in range(W):
            for a in range(A):
                s = 8 * (a + 1)
                anchors[i, j, a] = [j * 8, i * 8, j * 8 + s, i * 8 + s]
    rois, probs, n = V.generate_proposals(paddle.rand([1, A, H, W]),
                                          paddle.randn([1, 4 * A, H, W]) * 0.1,
                                          paddle.to_tensor(np.array([[32.0, 32.0]], np.float32)),
                                          paddle.to_tensor(anchors),
                                          paddle.to_tensor(np.ones_like(anchors)),
                                          pre_nms_top_n=30, post_nms_top_n=10,
                                          return_rois_num=True)
    assert rois.shape[0] == probs.shape[0] == int(n.numpy()[0]) <= 10


def test_read_decode_jpeg(tmp_path):
    from PIL import Image
    arr = (np.random.RandomState(0).rand(12, 10, 3) * 255).astype(np.uint8)
    p = str(tmp_path / 'a.jpg')
    Image.fromarray(arr).save(p, quality=95)
    data = V.read_file(p)
    assert data.dtype == paddle.uint8 and data.shape[0] > 100
    img = V.decode_jpeg(data)
    assert img.shape == [3, 12, 10]
    assert V.decode_jpeg(data, mode='gray').shape == [1, 12, 10]


def test_conv_norm_activation():
    blk = V.ConvNormActivation(3, 8, 3, stride=2)
    assert blk(paddle.randn([2, 3, 8, 8])).shape == [2, 8, 4, 4]
