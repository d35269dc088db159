"""Architecture facts of the reference ``CombinedModel`` and its state_dict layout.

Citations (reference = /root/reference):
  * trunk: torchvision resnet50 v1.5 via ``MultiTaskResNetFeatureExtractor``
    (training/modify_models.py:413-452) -> keys ``backbone.*``
  * YOLO branches: ``CustomYOLO`` adapter (modify_models.py:40-71) + YOLO v11n
    (training/yolopt/nets/nn.py:28-312) with the 1-class head swap (modify_models.py:156-180)
  * AdaFace: ``CustomAdaFace`` (modify_models.py:225-297) + IR-50
    (libs/net_adaface.py:144-167, 222-337) + AdaFace margin head (libs/head_adaface.py:45-70)
  * ViTPose: ``CustomVitPose`` (modify_models.py:348-385) + transformers ViTPose-B (simple decoder)

``state_dict_spec()`` returns [(key, shape, kind)] for the 2130 entries; it is checked
against the reference model's own ``state_dict()`` (keys and shapes recorded by
oracle/make_golden_evalsteps.py into tests/golden/sd_keys_ref.json) by
tests/test_abi_and_host.py::test_state_dict_spec_matches_reference_keys.
"""
from __future__ import annotations

# ----------------------------------------------------------------------------- IR-50
# (in_channel, depth, stride) per BasicBlockIR unit, libs/net_adaface.py:222-243
IR50_UNITS = []
for _cin, _d, _n in ((64, 64, 3), (64, 128, 4), (128, 256, 14), (256, 512, 3)):
    IR50_UNITS.append((_cin, _d, 2))
    IR50_UNITS += [(_d, _d, 1)] * (_n - 1)

# ResNet-50 stages: (planes, blocks, stride)
RESNET50_STAGES = ((64, 3, 1), (128, 4, 2), (256, 6, 2), (512, 3, 2))

YOLO_WIDTH = (3, 16, 32, 64, 128, 256)
VIT_HIDDEN, VIT_LAYERS, VIT_HEADS, VIT_MLP = 768, 12, 12, 3072
VIT_IMG = (256, 192)
VIT_PATCH = 16
VIT_GRID = (16, 12)          # (256+4-16)//16+1, (192+4-16)//16+1  (patch conv pad 2)
NUM_KEYPOINTS = 17
HEATMAP = (64, 48)
ADAFACE_CLASSES = 85742

TASKS = ("face_detection", "person_detection", "pose_estimation", "face_recognition")


class _Spec:
    def __init__(self):
        self.items = []

    def add(self, name, shape, kind):
        self.items.append((name, tuple(shape), kind))

    def conv(self, name, co, ci, k, bias=False, groups=1):
        self.add(name + ".weight", (co, ci // groups, k, k), "conv")
        if bias:
            self.add(name + ".bias", (co,), "bias")

    def linear(self, name, co, ci, bias=True):
        self.add(name + ".weight", (co, ci), "linear")
        if bias:
            self.add(name + ".bias", (co,), "bias")

    def bn(self, name, c, affine=True):
        if affine:
            self.add(name + ".weight", (c,), "bn")
            self.add(name + ".bias", (c,), "bn")
        self.add(name + ".running_mean", (c,), "bn")
        self.add(name + ".running_var", (c,), "bn")
        self.add(name + ".num_batches_tracked", (), "bn")

    def prelu(self, name, c):
        self.add(name + ".weight", (c,), "prelu")

    def ln(self, name, c):
        self.add(name + ".weight", (c,), "ln")
        self.add(name + ".bias", (c,), "ln")

    # YOLO ``Conv`` block: conv (no bias) + BN(eps 1e-3) + act   (nn.py:28-39)
    def yconv(self, name, ci, co, k, g=1):
        self.conv(name + ".conv", co, ci, k, groups=g)
        self.bn(name + ".norm", co)


def _residual(s, p, ch, e):
    s.yconv(p + ".conv1", ch, int(ch * e), 3)
    s.yconv(p + ".conv2", int(ch * e), ch, 3)


def _cspmodule(s, p, cin, cout):
    s.yconv(p + ".conv1", cin, cout // 2, 1)
    s.yconv(p + ".conv2", cin, cout // 2, 1)
    s.yconv(p + ".conv3", 2 * (cout // 2), cout, 1)
    _residual(s, p + ".res_m.0", cout // 2, 1.0)
    _residual(s, p + ".res_m.1", cout // 2, 1.0)


def _csp(s, p, cin, cout, n, csp, r):
    s.yconv(p + ".conv1", cin, 2 * (cout // r), 1)
    s.yconv(p + ".conv2", (2 + n) * (cout // r), cout, 1)
    for i in range(n):
        if csp:
            _cspmodule(s, f"{p}.res_m.{i}", cout // r, cout // r)
        else:
            _residual(s, f"{p}.res_m.{i}", cout // r, 0.5)


def _psa(s, p, ch, n):
    s.yconv(p + ".conv1", ch, 2 * (ch // 2), 1)
    s.yconv(p + ".conv2", 2 * (ch // 2), ch, 1)
    c = ch // 2
    nh = ch // 128                    # PSABlock(ch // 2, ch // 128), nn.py:144
    dk = (c // nh) // 2
    for i in range(n):
        b = f"{p}.res_m.{i}"
        s.yconv(b + ".conv1.qkv", c, c + dk * nh * 2, 1)
        s.yconv(b + ".conv1.conv1", c, c, 3, g=c)
        s.yconv(b + ".conv1.conv2", c, c, 1)
        s.yconv(b + ".conv2.0", c, 2 * c, 1)
        s.yconv(b + ".conv2.1", 2 * c, c, 1)


def _yolo_branch(s, p):
    a = p + ".adapter"
    s.conv(a + ".0", 512, 2048, 1, bias=True); s.bn(a + ".1", 512)
    s.conv(a + ".4", 512, 512, 3, bias=True); s.bn(a + ".5", 512)
    s.conv(a + ".7", 256, 512, 1, bias=True); s.bn(a + ".8", 256)
    s.conv(a + ".10", 128, 256, 3, bias=True); s.bn(a + ".11", 128)
    s.conv(a + ".13", 64, 128, 1, bias=True); s.bn(a + ".14", 64)
    s.conv(a + ".16", 3, 64, 3, bias=True); s.bn(a + ".17", 3)
    w = YOLO_WIDTH
    n = p + ".yolo.net"
    s.yconv(n + ".p1.0", w[0], w[1], 3)
    s.yconv(n + ".p2.0", w[1], w[2], 3); _csp(s, n + ".p2.1", w[2], w[3], 1, False, 4)
    s.yconv(n + ".p3.0", w[3], w[3], 3); _csp(s, n + ".p3.1", w[3], w[4], 1, False, 4)
    s.yconv(n + ".p4.0", w[4], w[4], 3); _csp(s, n + ".p4.1", w[4], w[4], 1, True, 2)
    s.yconv(n + ".p5.0", w[4], w[5], 3); _csp(s, n + ".p5.1", w[5], w[5], 1, True, 2)
    s.yconv(n + ".p5.2.conv1", w[5], w[5] // 2, 1); s.yconv(n + ".p5.2.conv2", w[5] * 2, w[5], 1)
    _psa(s, n + ".p5.3", w[5], 1)
    f = p + ".yolo.fpn"
    _csp(s, f + ".h1", w[4] + w[5], w[4], 1, False, 2)
    _csp(s, f + ".h2", w[4] + w[4], w[3], 1, False, 2)
    s.yconv(f + ".h3", w[3], w[3], 3)
    _csp(s, f + ".h4", w[3] + w[4], w[4], 1, False, 2)
    s.yconv(f + ".h5", w[4], w[4], 3)
    _csp(s, f + ".h6", w[4] + w[5], w[5], 1, True, 2)
    h = p + ".yolo.head"
    s.add(h + ".dfl.conv.weight", (1, 16, 1, 1), "other")
    for i, x in enumerate((w[3], w[4], w[5])):
        s.yconv(f"{h}.box.{i}.0", x, 64, 3)
        s.yconv(f"{h}.box.{i}.1", 64, 64, 3)
        s.conv(f"{h}.box.{i}.2", 64, 64, 1, bias=True)
    for i, x in enumerate((w[3], w[4], w[5])):
        s.yconv(f"{h}.cls.{i}.0", x, x, 3, g=x)
        s.yconv(f"{h}.cls.{i}.1", x, 80, 1)
        s.yconv(f"{h}.cls.{i}.2", 80, 80, 3, g=80)
        s.yconv(f"{h}.cls.{i}.3", 80, 80, 1)
        s.conv(f"{h}.cls.{i}.4", 1, 80, 1, bias=True)


def state_dict_spec():
    s = _Spec()
    # trunk
    s.conv("backbone.conv1", 64, 3, 7); s.bn("backbone.bn1", 64)
    inpl = 64
    for li, (planes, blocks, stride) in enumerate(RESNET50_STAGES, 1):
        for b in range(blocks):
            p = f"backbone.layer{li}.{b}"
            s.conv(p + ".conv1", planes, inpl, 1); s.bn(p + ".bn1", planes)
            s.conv(p + ".conv2", planes, planes, 3); s.bn(p + ".bn2", planes)
            s.conv(p + ".conv3", planes * 4, planes, 1); s.bn(p + ".bn3", planes * 4)
            if b == 0:
                s.conv(p + ".downsample.0", planes * 4, inpl, 1); s.bn(p + ".downsample.1", planes * 4)
            inpl = planes * 4
    _yolo_branch(s, "yolo_face")
    _yolo_branch(s, "yolo_person")
    # AdaFace
    a = "ada_face.adapter"
    s.conv(a + ".0", 512, 2048, 1, bias=True); s.bn(a + ".1", 512); s.prelu(a + ".2", 512)
    s.conv(a + ".4", 256, 512, 3, bias=True); s.bn(a + ".5", 256); s.prelu(a + ".6", 256)
    s.conv(a + ".7", 128, 256, 3, bias=True); s.bn(a + ".8", 128); s.prelu(a + ".9", 128)
    s.conv(a + ".10", 64, 128, 3, bias=True); s.bn(a + ".11", 64); s.prelu(a + ".12", 64)
    m = "ada_face.adaface_model"
    s.conv(m + ".input_layer.0", 64, 64, 3); s.bn(m + ".input_layer.1", 64); s.prelu(m + ".input_layer.2", 64)
    s.bn(m + ".output_layer.0", 512)
    s.linear(m + ".output_layer.3", 512, 512 * 7 * 7)
    s.bn(m + ".output_layer.4", 512, affine=False)
    for i, (cin, d, st) in enumerate(IR50_UNITS):
        p = f"{m}.body.{i}"
        if cin != d:
            s.conv(p + ".shortcut_layer.0", d, cin, 1); s.bn(p + ".shortcut_layer.1", d)
        s.bn(p + ".res_layer.0", cin)
        s.conv(p + ".res_layer.1", d, cin, 3); s.bn(p + ".res_layer.2", d); s.prelu(p + ".res_layer.3", d)
        s.conv(p + ".res_layer.4", d, d, 3); s.bn(p + ".res_layer.5", d)
    s.add("ada_face.head.kernel", (512, ADAFACE_CLASSES), "other")
    s.add("ada_face.head.t", (1,), "other")
    s.add("ada_face.head.batch_mean", (1,), "other")
    s.add("ada_face.head.batch_std", (1,), "other")
    # ViTPose
    a = "vit_pose.adapter"
    s.conv(a + ".0", 512, 2048, 1, bias=True); s.bn(a + ".1", 512)
    s.conv(a + ".4", 256, 512, 3, bias=True); s.bn(a + ".5", 256)
    s.conv(a + ".7", 128, 256, 3, bias=True); s.bn(a + ".8", 128)
    s.conv(a + ".10", 3, 128, 3, bias=True); s.bn(a + ".11", 3)
    v = "vit_pose.vit_pose.backbone"
    s.add(v + ".embeddings.position_embeddings", (1, VIT_GRID[0] * VIT_GRID[1] + 1, VIT_HIDDEN), "other")
    s.conv(v + ".embeddings.patch_embeddings.projection", VIT_HIDDEN, 3, VIT_PATCH, bias=True)
    for i in range(VIT_LAYERS):
        L = f"{v}.encoder.layer.{i}"
        for q in ("query", "key", "value"):
            s.linear(f"{L}.attention.attention.{q}", VIT_HIDDEN, VIT_HIDDEN)
        s.linear(L + ".attention.output.dense", VIT_HIDDEN, VIT_HIDDEN)
        s.linear(L + ".mlp.fc1", VIT_MLP, VIT_HIDDEN)
        s.linear(L + ".mlp.fc2", VIT_HIDDEN, VIT_MLP)
        s.ln(L + ".layernorm_before", VIT_HIDDEN)
        s.ln(L + ".layernorm_after", VIT_HIDDEN)
    s.ln(v + ".layernorm", VIT_HIDDEN)
    s.conv("vit_pose.vit_pose.head.conv", NUM_KEYPOINTS, VIT_HIDDEN, 3, bias=True)
    return s.items
