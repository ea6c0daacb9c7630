from .layers import Layer, ParamAttr, WeightNormParamAttr  # noqa
from .common import *  # noqa
from .norm import *  # noqa
from .conv import *  # noqa
from .loss import *  # noqa
from .transformer import *  # noqa
from .rnn import *  # noqa
