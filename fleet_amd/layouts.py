"""Gradient upload layouts of the reference's cppNN models.

An upload is ``Base64::encode(cnn.gradients())`` (Client/app/src/main/cpp/
cppNN-lib.cpp:218-234) with ``gradients()`` = [nW, (size_i, dW_i...)*, nB,
(size_j, db_j...)*] (commonLib/cppNN/network.h:1038-1056): one weight block per
layer-graph edge and one bias block per layer.

* MNIST: the network built in Driver/src/main/c++/cppNN_backend.cpp:109-117
  (I1 28x28x1, C1 conv5x8, P1 pool3, C2i conv1x16, C2 conv5x48, P2 pool2, FC2 softmax10).
* CIFAR-10/100: the commented architecture at Driver/src/main/c++/cppNN_backend.cpp:121-136
  (I1 32x32x3, C1 conv3x16, P1 maxpool3/2, C2 conv3x64, P2 maxpool4/4, FC384, FC192, softmax 10/100).
* synthetic: one weight block and no bias block, [1, N, x..., 0], sized so the
  upload holds exactly the stated number of floats.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Tuple


@dataclass(frozen=True)
class Layout:
    name: str
    w_sizes: Tuple[int, ...]
    b_sizes: Tuple[int, ...]
    # layers whose update_bias is not the base no-op (fully_connected_layer,
    # commonLib/cppNN/layer.h:241-243): the biases descentNative updates
    fc_layers: Tuple[int, ...] = ()

    def w_present(self):
        """W slot non-null (a weight block of size 0 is a layer-graph edge without
        weights, e.g. into a pooling layer)."""
        return tuple(s > 0 for s in self.w_sizes)

    def fc_flags(self):
        return tuple(k in self.fc_layers for k in range(len(self.b_sizes)))

    @property
    def n_weights(self) -> int:
        return sum(self.w_sizes)

    @property
    def n_fc_bias(self) -> int:
        return sum(self.b_sizes[k] for k in self.fc_layers)

    @property
    def n_up(self) -> int:
        return 2 + len(self.w_sizes) + len(self.b_sizes) + sum(self.w_sizes) + sum(self.b_sizes)

    @property
    def n_flat(self) -> int:
        return sum(self.w_sizes) + sum(self.b_sizes)

    def header_positions(self):
        pos, idx = [], 0
        pos.append(idx)
        idx += 1
        for s in self.w_sizes:
            pos.append(idx)
            idx += 1 + s
        pos.append(idx)
        idx += 1
        for s in self.b_sizes:
            pos.append(idx)
            idx += 1 + s
        return pos

    def header_values(self):
        vals = [float(len(self.w_sizes))] + [float(s) for s in self.w_sizes]
        vals += [float(len(self.b_sizes))] + [float(s) for s in self.b_sizes]
        return vals


def synthetic(n_up: int) -> Layout:
    """[1, N, x_0..x_{N-1}, 0] with N = n_up - 3 (one weight block, no biases)."""
    return Layout(f"synthetic{n_up}", (n_up - 3,), ())


MNIST = Layout("mnist", (200, 0, 128, 19200, 0, 1920), (784, 0, 512, 0, 0, 192, 10), (6,))
CIFAR10 = Layout("cifar10", (432, 0, 9216, 0, 221184, 73728, 1920), (3072, 0, 3136, 0, 576, 384, 192, 10),
                 (5, 6, 7))
CIFAR100 = Layout("cifar100", (432, 0, 9216, 0, 221184, 73728, 19200), (3072, 0, 3136, 0, 576, 384, 192, 100),
                  (5, 6, 7))

LAYOUTS = {
    "mnist": MNIST,
    "cifar10": CIFAR10,
    "cifar100": CIFAR100,
    "synth1m": synthetic(1 << 20),
    # configs[4]'s 4,194,304 values as two weight blocks, [2, N1, x.., N2, y.., 0]: one block
    # of N = 4,194,301 does not survive the codec (N * 10^2 is no binary32 value; it decodes
    # to 4194300.75, so the reference's flatGrad walk would read a payload slot as the bias
    # count), while N1 = 2^21 and N2 = 2,097,148 (multiples of 4) round-trip exactly
    "synth4m": Layout("synth4m", (1 << 21, (1 << 22) - 4 - (1 << 21)), ()),
}

assert MNIST.n_up == 22961 and CIFAR10.n_up == 313867 and CIFAR100.n_up == 331237
