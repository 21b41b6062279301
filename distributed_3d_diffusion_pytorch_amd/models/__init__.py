from .xunet import (XUNet, ResnetBlock, AttnBlock, AttnLayer, XUNetBlock, ConditioningProcessor, FiLM,
                    GroupNorm, count_params)
from .reference import reference_forward, reference_forward_grad

__all__ = ["XUNet", "ResnetBlock", "AttnBlock", "AttnLayer", "XUNetBlock", "ConditioningProcessor", "FiLM",
           "GroupNorm", "count_params", "reference_forward", "reference_forward_grad"]
