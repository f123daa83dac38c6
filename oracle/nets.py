"""TF1 numerics of the MADDPG trainer, restated in numpy fp32 (test oracle).

* ``mlp_fwd``/``mlp_bwd``: ``experiments/train.py:39-46`` -- three
  ``fully_connected`` layers (ReLU, ReLU, linear), W stored [in, out].
* ``gumbel_softmax``: ``SoftCategoricalPd.sample`` (``distributions.py:264-266``)
  ``softmax(logits - log(-log(u)))`` with injected uniforms ``u``.
* ``clip_by_norm``: TF1 ``clip_ops.clip_by_norm`` as used per tensor by
  ``tf_util.minimize_and_clip`` (``tf_util.py:177-180``):
  ``(g * c) / max(sqrt(sum(g*g)), c)``.
* ``adam_apply``: TF1 ``ApplyAdam`` (training_ops.cc), fp32, no FMA:
  ``alpha = lr*sqrt(1-b2^t)/(1-b1^t); m += (g-m)*(1-b1); v += (g*g-v)*(1-b2);
  var -= (m*alpha)/(sqrt(v)+eps)``; beta powers are fp32 variables
  initialised to b1/b2 and multiplied after every apply (``AdamOptimizer._finish``).
* ``polyak``: ``make_update_exp`` (``maddpg.py:20-26``):
  ``t = 0.99f*t + 0.01f*v``.
"""
import numpy as np

F32 = np.float32
NAMES = ("W1", "b1", "W2", "b2", "W3", "b3")


def xavier_init(rng, n_in, n_out, units):
    """tf.contrib.layers.fully_connected default init (xavier uniform W, zero b)."""
    def w(a, b):
        lim = np.sqrt(6.0 / (a + b))
        return rng.uniform(-lim, lim, size=(a, b)).astype(F32)
    return {
        "W1": w(n_in, units), "b1": np.zeros(units, F32),
        "W2": w(units, units), "b2": np.zeros(units, F32),
        "W3": w(units, n_out), "b3": np.zeros(n_out, F32),
    }


def relu(x):
    return np.maximum(x, F32(0))


def mlp_fwd(p, x):
    x = x.astype(F32)
    h1 = relu(x @ p["W1"] + p["b1"])
    h2 = relu(h1 @ p["W2"] + p["b2"])
    y = h2 @ p["W3"] + p["b3"]
    return y, (x, h1, h2)


def mlp_bwd(p, cache, dy, need_dx=False):
    """Gradients of sum(dy * y) w.r.t. all params (and x). ReLU grad uses out>0."""
    x, h1, h2 = cache
    dy = dy.astype(F32)
    g = {"W3": h2.T @ dy, "b3": dy.sum(0)}
    dh2 = (dy @ p["W3"].T) * (h2 > 0)
    g["W2"] = h1.T @ dh2
    g["b2"] = dh2.sum(0)
    dh1 = (dh2 @ p["W2"].T) * (h1 > 0)
    g["W1"] = x.T @ dh1
    g["b1"] = dh1.sum(0)
    g = {k: v.astype(F32) for k, v in g.items()}
    if need_dx:
        return g, (dh1 @ p["W1"].T).astype(F32)
    return g


def input_grad(p, cache, dy):
    """d(sum(dy*y))/dx only (no weight grads)."""
    x, h1, h2 = cache
    dh2 = (dy.astype(F32) @ p["W3"].T) * (h2 > 0)
    dh1 = (dh2 @ p["W2"].T) * (h1 > 0)
    return (dh1 @ p["W1"].T).astype(F32)


def softmax(z):
    z = z - z.max(axis=-1, keepdims=True)
    e = np.exp(z)
    return (e / e.sum(axis=-1, keepdims=True)).astype(F32)


def gumbel_softmax(logits, u):
    """distributions.py:264-266 with injected u ~ U[0,1) (fp32)."""
    with np.errstate(divide="ignore"):
        z = logits.astype(F32) - np.log(-np.log(u.astype(F32)))
    return softmax(z)


def softmax_bwd(a, da):
    """TF SoftmaxGrad: (da - sum(da*a)) * a."""
    return ((da - (da * a).sum(-1, keepdims=True)) * a).astype(F32)


# How clip_by_norm takes the tensor norm.  "fp32" (default, tf_util.py:178-180
# through TF1's clip_ops.clip_by_norm): l2norm = sqrt(reduce_sum(t * t)) with
# t * t and the sum in fp32 -- the reference's own arithmetic (numpy's pairwise
# order stands in for Eigen's, which no restatement reproduces bit for bit).
# "fp64": the sum of squares in float64, rounded to fp32 after the sqrt -- the
# value every fp32 summation order approximates, and what the device optimizer
# computes (fp64 per-chunk sums combined in chunk order, so every split of a
# tensor into chunks and every replica agrees).  tests/test_gpu_parity.py
# reports the device's distance to both (the two norms differ by <= ~1e-7
# relative; Adam's step barely sees a common scale of its gradient).
CLIP_NORM = "fp32"


def tensor_norm(g, mode=None):
    mode = mode or CLIP_NORM
    if mode == "fp32":
        g32 = g.astype(F32)
        return np.sqrt(np.sum(g32 * g32, dtype=F32)).astype(F32)
    return np.sqrt(np.sum(g.astype(np.float64) ** 2)).astype(F32)


def clip_by_norm(g, c=0.5, mode=None):
    """tf_util.py:178-180: (g * c) / max(||g||, c), per tensor."""
    c = F32(c)
    n = tensor_norm(g, mode)
    return ((g * c) / np.maximum(n, c)).astype(F32)


class Adam:
    """One TF1 AdamOptimizer (own beta powers) over a dict of tensors."""

    def __init__(self, params, lr=1e-2, b1=0.9, b2=0.999, eps=1e-8):
        self.lr, self.b1, self.b2, self.eps = F32(lr), F32(b1), F32(b2), F32(eps)
        self.m = {k: np.zeros_like(v) for k, v in params.items()}
        self.v = {k: np.zeros_like(v) for k, v in params.items()}
        self.b1p = F32(b1)
        self.b2p = F32(b2)

    def apply(self, params, grads):
        one = F32(1)
        alpha = F32(self.lr * np.sqrt(one - self.b2p) / (one - self.b1p))
        for k in params:
            g = grads[k]
            m = self.m[k] + (g - self.m[k]) * (one - self.b1)
            v = self.v[k] + (g * g - self.v[k]) * (one - self.b2)
            params[k] = (params[k] - (m * alpha) / (np.sqrt(v) + self.eps)).astype(F32)
            self.m[k], self.v[k] = m.astype(F32), v.astype(F32)
        self.b1p = F32(self.b1p * self.b1)
        self.b2p = F32(self.b2p * self.b2)


def polyak(target, online, tau=1e-2):
    """maddpg.py:20-26: polyak = 1 - 1e-2, fp32 constants."""
    a = F32(1.0 - tau)
    b = F32(1.0 - (1.0 - tau))
    for k in target:
        target[k] = (a * target[k] + b * online[k]).astype(F32)
