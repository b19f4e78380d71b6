"""Autograd references of the framework's models built from plain PyTorch ops, sharing the
model's parameter tensors. Used to check the hand-written backward passes."""
import torch
import torch.nn.functional as F


def conv_ref(layer, x, params):
    s = layer.spec
    w = params[layer.w.name].permute(0, 3, 1, 2)
    xt = F.pad(x, (s.pl, s.pr, s.pt, s.pb))
    return F.conv2d(xt, w, stride=(s.sh, s.sw), dilation=(s.dh, s.dw))


def convbn_ref(layer, x, params, residual=None):
    z = conv_ref(layer, x, params)
    if layer.bn:
        z = F.batch_norm(z, None, None, params[layer.gamma.name], params[layer.beta.name], training=True,
                         eps=layer.eps)
    if residual is not None:
        z = z + residual
    if layer.relu:
        z = torch.relu(z)
    return z


def pool_ref(layer, x):
    pt, pb, pl, pr = layer.pads
    if layer.is_max:
        return F.max_pool2d(F.pad(x, (pl, pr, pt, pb), value=-float("inf")), layer.k, layer.s)
    if layer.incl_pad:
        return F.avg_pool2d(F.pad(x, (pl, pr, pt, pb)), layer.k, layer.s)
    ones = torch.ones_like(x[:, :1])
    s = F.avg_pool2d(F.pad(x, (pl, pr, pt, pb)), layer.k, layer.s, divisor_override=1)
    c = F.avg_pool2d(F.pad(ones, (pl, pr, pt, pb)), layer.k, layer.s, divisor_override=1)
    return s / c


def resnet_ref(model, images_nhwc, params):
    x = images_nhwc.permute(0, 3, 1, 2)
    x = convbn_ref(model.stem, x, params)
    x = pool_ref(model.pool, x)
    for b in model.blocks:
        sc = convbn_ref(b.sc, x, params) if b.proj else x
        a = convbn_ref(b.c1, x, params)
        a = convbn_ref(b.c2, a, params)
        x = convbn_ref(b.c3, a, params, residual=sc)
    feat = x.mean(dim=(2, 3))
    w = params[model.fc.w.name].view(model.fc.ncls, -1)
    return feat @ w.t() + params[model.fc.b.name]


def reference_grads(model, images, labels, ref_fn):
    params = {p.name: p.data.detach().clone().to(images.dtype).requires_grad_(True) for p in model.ps.params}
    logits = ref_fn(model, images, params)
    loss = F.cross_entropy(logits, labels)
    loss.backward()
    return loss.detach(), {k: v.grad for k, v in params.items()}, logits.detach()


def _gamma(layer, params):
    name = getattr(layer.gamma, "name", None)
    return params[name] if name in params else layer.gamma.data.to(next(iter(params.values())).dtype)


def convbn_ref2(layer, x, params, residual=None):
    """convbn_ref that also handles BN(scale=False) layers (fixed gamma)."""
    z = conv_ref(layer, x, params)
    z = F.batch_norm(z, None, None, _gamma(layer, params), params[layer.beta.name], training=True, eps=layer.eps)
    if residual is not None:
        z = z + residual
    if layer.relu:
        z = torch.relu(z)
    return z


def _layer_ref(layer, x, params):
    from azure_hc_intel_tf_amd.nn.layers import ConvBN

    if isinstance(layer, ConvBN):
        return convbn_ref2(layer, x, params)
    return pool_ref(layer, x)


def inception_ref(model, images_nhwc, params):
    x = images_nhwc.permute(0, 3, 1, 2)
    for l in model.stem:
        x = _layer_ref(l, x, params)
    for m in model.modules:
        outs = {}
        for n in m.nodes:
            inp = x if n.src is None else outs[id(n.src)]
            outs[id(n)] = _layer_ref(n.layer, inp, params)
        x = torch.cat([outs[id(t)] for t in m.terminals], dim=1)
    feat = x.mean(dim=(2, 3))
    w = params[model.fc.w.name].view(model.fc.ncls, -1)
    return feat @ w.t() + params[model.fc.b.name]
