"""Drop-in BO drivers: MultiSurrogateOptimiser, MonoSurrogateOptimiser, EMO, ParEGO."""
from .emo import EMO
from .optimisers import MonoSurrogateOptimiser, MultiSurrogateOptimiser
from .parego import ParEGO

__all__ = ["MultiSurrogateOptimiser", "MonoSurrogateOptimiser", "EMO", "ParEGO"]
