from .raft import RAFT
from .corr import CorrBlock, AlternateCorrBlock
from .extractor import BasicEncoder, SmallEncoder, ResidualBlock, BottleneckBlock
from .update import (BasicUpdateBlock, SmallUpdateBlock, SepConvGRU, ConvGRU, FlowHead,
                     BasicMotionEncoder, SmallMotionEncoder)
