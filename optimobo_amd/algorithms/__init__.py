"""Drop-in BO drivers: MultiSurrogateOptimiser, MonoSurrogateOptimiser, EMO, ParEGO, KEEP, TuRBO_1, TuRBO_M."""
from .emo import EMO
from .keep import KEEP
from .optimisers import MonoSurrogateOptimiser, MultiSurrogateOptimiser
from .parego import ParEGO
from .turbo import TuRBO_1, TuRBO_M

__all__ = ["MultiSurrogateOptimiser", "MonoSurrogateOptimiser", "EMO", "ParEGO", "KEEP", "TuRBO_1", "TuRBO_M"]
