"""Kernel identity on the Python side of the boundary.

Restates the reference's kernel string format and factory
(`KernelFactory<T>::GetKernel`, include/KernelFactory.h:83-178; leaf `ToString` via
`Kernel::ParametersToString`, include/Kernel.h:75-82) and lowers a kernel tree into the
post-order `gprx_kernel_desc` program of include/gprx.h.
"""
from dataclasses import dataclass, field
from typing import List, Optional

OP = {
    "GaussianKernel": 1,
    "GaussianExpKernel": 2,
    "WhiteKernel": 3,
    "RationalQuadraticKernel": 4,
    "PeriodicKernel": 5,
    "SumKernel": 6,
    "ProductKernel": 7,
}
NPARAMS = {"GaussianKernel": 2, "GaussianExpKernel": 2, "WhiteKernel": 1, "RationalQuadraticKernel": 3,
           "PeriodicKernel": 3}


class KernelError(ValueError):
    pass


@dataclass
class KernelNode:
    name: str
    params: List[float] = field(default_factory=list)
    k1: Optional["KernelNode"] = None
    k2: Optional["KernelNode"] = None

    @property
    def is_leaf(self):
        return self.name not in ("SumKernel", "ProductKernel")

    def num_params(self):
        if self.is_leaf:
            return NPARAMS[self.name]
        return self.k1.num_params() + self.k2.num_params()

    def parameters(self):
        """GetParameters() order (include/Kernel.h:187-193, 336-340)."""
        if self.is_leaf:
            return list(self.params)
        return self.k1.parameters() + self.k2.parameters()

    def to_string(self, digits=16):
        """ToString() (include/Kernel.h:198-200, 497-499): leaf params each followed by ','."""
        if self.is_leaf:
            body = "".join(f"{p:.{digits}g}," for p in self.params)
            return f"{self.name}({body})"
        return f"{self.name}({self.k1.to_string(digits)},{self.k2.to_string(digits)})"

    def postorder(self):
        if self.is_leaf:
            return [(OP[self.name], list(self.params))]
        return self.k1.postorder() + self.k2.postorder() + [(OP[self.name], [])]


def Gaussian(sigma, scale=1.0):
    return KernelNode("GaussianKernel", [float(sigma), float(scale)])


def GaussianExp(sigma, scale=1.0):
    return KernelNode("GaussianExpKernel", [float(sigma), float(scale)])


def White(scale):
    return KernelNode("WhiteKernel", [float(scale)])


def RationalQuadratic(scale, sigma, alpha):
    return KernelNode("RationalQuadraticKernel", [float(scale), float(sigma), float(alpha)])


def Periodic(scale, b, sigma):
    return KernelNode("PeriodicKernel", [float(scale), float(b), float(sigma)])


def Sum(k1, k2):
    return KernelNode("SumKernel", k1=k1, k2=k2)


def Product(k1, k2):
    return KernelNode("ProductKernel", k1=k1, k2=k2)


class _Cursor:
    def __init__(self, s):
        self.s = s


def _parse(cur: _Cursor) -> KernelNode:
    # include/KernelFactory.h:83-178 — the remaining string is consumed by reference
    s = cur.s
    p = s.find("(")
    if p < 0:
        raise KernelError("KernelFactory::GetKernel: failed to tokanize kernel name string")
    name = s[:p]
    if name in ("SumKernel", "ProductKernel"):
        cur.s = s[len(name) + 1:]
        k1 = _parse(cur)
        pos = cur.s.find("),")
        if pos < 0:
            raise KernelError(f"KernelFactory::GetKernel: failed to tokanize  {name} name string")
        cur.s = cur.s[pos + 2:]
        k2 = _parse(cur)
        return KernelNode(name, k1=k1, k2=k2)
    rest = s[p + 1:]
    params = []
    for tok in rest.split(","):
        if ")" in tok:
            break
        params.append(tok)
    if name not in NPARAMS:
        raise KernelError("KernelFactory::GetKernel: failed to load kernel.")
    if len(params) != NPARAMS[name]:
        raise KernelError(f"{name}::Load: wrong number of kernel parameters.")
    vals = [float(x) for x in params]
    node = KernelNode(name, vals)
    validate(node)
    return node


def validate(node: KernelNode):
    """Constructor-time parameter checks (include/Kernel.h:529-530, 1003-1005)."""
    if node.name == "GaussianKernel":
        if node.params[0] == 0:
            raise KernelError("GaussianKernel: sigma has to be positive")
        if node.params[1] == 0:
            raise KernelError("GaussianKernel: scale has to be positive")
    if node.name == "PeriodicKernel":
        if node.params[0] == 0:
            raise KernelError("PeriodicKernel: scale parameter has to be positive.")
        if node.params[1] == 0:
            raise KernelError("PeriodicKernel: period length parameter has to be positive.")
        if node.params[2] == 0:
            raise KernelError("PeriodicKernel: sigma parameter has to be positive.")


def parse_kernel(s: str) -> KernelNode:
    return _parse(_Cursor(s))


def as_node(k) -> KernelNode:
    if isinstance(k, KernelNode):
        return k
    if isinstance(k, str):
        return parse_kernel(k)
    raise TypeError(k)


def general_kernel(p):
    """KernelUtils GetGeneralKernel (include/KernelUtils.h:43-89) from 13 parameters:
    Sum(Sum(Sum(G(sigma=p1,scale=p0), Product(G(p3,p2), P(p4,p5,p6))), RQ(p7,p8,p9)),
        Sum(G(p11,p10), W(p12)))  — note the (scale, sigma) order of the Gaussian inputs."""
    if len(p) != 13:
        raise KernelError("GetGeneralKernel: 13 parameters required")
    g1 = Gaussian(p[1], p[0])
    gp = Product(Gaussian(p[3], p[2]), Periodic(p[4], p[5], p[6]))
    rq = RationalQuadratic(p[7], p[8], p[9])
    gw = Sum(Gaussian(p[11], p[10]), White(p[12]))
    return Sum(Sum(Sum(g1, gp), rq), gw)
