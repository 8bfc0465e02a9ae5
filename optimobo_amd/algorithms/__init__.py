"""Drop-in BO drivers: MultiSurrogateOptimiser, MonoSurrogateOptimiser, EMO, ParEGO, ParEGO_C1/C2, KEEP,
TuRBO_1, TuRBO_M."""
from .cparego import ParEGO_C1, ParEGO_C2
from .emo import EMO
from .keep import KEEP
from .optimisers import MonoSurrogateOptimiser, MultiSurrogateOptimiser
from .parego import ParEGO
from .turbo import TuRBO_1, TuRBO_M

__all__ = ["MultiSurrogateOptimiser", "MonoSurrogateOptimiser", "EMO", "ParEGO", "ParEGO_C1", "ParEGO_C2", "KEEP",
           "TuRBO_1", "TuRBO_M"]
