"""Activation functions (mirrors skge/actfun.py).  ``code`` is the id the HIP
kernels use (include/skge_hip.h SKGE_AF_*); f / g_given_f are kept on the
host for API compatibility."""
import numpy as np

from . import _lib as L


class ActivationFunction(object):
    code = None

    @classmethod
    def key(cls):
        return cls.__name__.lower()


class Linear(ActivationFunction):
    """skge/actfun.py:13-24"""
    code = L.SKGE_AF_LINEAR

    @staticmethod
    def f(x):
        return x

    @staticmethod
    def g_given_f(fx):
        return np.ones(fx.shape[0])


class Sigmoid(ActivationFunction):
    """skge/actfun.py:27-35"""
    code = L.SKGE_AF_SIGMOID

    @staticmethod
    def f(x):
        return 1.0 / (1 + np.exp(-x))

    @staticmethod
    def g_given_f(fx):
        return fx * (1.0 - fx)


class Tanh(ActivationFunction):
    """skge/actfun.py:38-46"""
    code = L.SKGE_AF_TANH

    @staticmethod
    def f(x):
        return np.tanh(x)

    @staticmethod
    def g_given_f(fx):
        return 1 - fx ** 2


class ReLU(ActivationFunction):
    """skge/actfun.py:49-57"""
    code = L.SKGE_AF_RELU

    @staticmethod
    def f(x):
        return np.maximum(0, x)

    @staticmethod
    def g_given_f(fx):
        return np.int_(fx > 0)


class Softplus(ActivationFunction):
    """skge/actfun.py:60-68 (no gradient in the reference either)."""

    @staticmethod
    def f(x):
        return np.log(1 + np.exp(x))

    @staticmethod
    def g(x):
        raise NotImplementedError()


afuns = {}
for cls in ActivationFunction.__subclasses__():
    afuns[cls.key()] = cls


def af_code(af):
    if isinstance(af, str):
        af = afuns[af]
    if af.code is None:
        raise ValueError("activation %s has no gradient (skge/actfun.py:60-68)" % af.key())
    return af.code
