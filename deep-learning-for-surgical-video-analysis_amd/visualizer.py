"""Top-level ``visualizer`` module kept so ``from visualizer import get_local`` resolves
(mix_transformer_evp.py:69).  The reference's ``get_local`` rewrites a function's bytecode to
capture a local (the attention map) when activated (visualizer.py:10-33); the MI355X
attention kernel never materialises that map, so activation is refused loudly."""


class get_local(object):
    cache = {}
    is_activate = False

    def __init__(self, varname):
        self.varname = varname

    def __call__(self, func):
        if type(self).is_activate:
            raise NotImplementedError("get_local: attention-map capture is not available on the svk path "
                                      "(the fused attention kernel does not materialise attn)")
        return func

    @classmethod
    def clear(cls):
        for key in cls.cache.keys():
            cls.cache[key] = []

    @classmethod
    def activate(cls):
        cls.is_activate = True
