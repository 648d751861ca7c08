"""Framework dispatch (models/frameworks/__init__.py:1-10)."""


def get_model(args):
    from ..config import as_cfg
    args = as_cfg(args)
    fw = args.model.framework
    if fw == 'NeuS':
        from .neus import get_model as gm
    elif fw == 'VolSDF':
        from .volsdf import get_model as gm
    elif fw == 'UNISURF':
        from .unisurf import get_model as gm
    else:
        raise NotImplementedError(fw)
    return gm(args)
