"""Importance-sampling core: pool sampler math, global-table sampler, alias tables."""
from .pool import (cumulative_means, ema_replay, importance_probs, draw, is_weights,
                   weighted_loss, score_and_sample)
from .groupwise import Groupwise_Sampler
from .alias import build_alias, alias_draw, alias_distribution

__all__ = ['cumulative_means', 'ema_replay', 'importance_probs', 'draw', 'is_weights',
           'weighted_loss', 'score_and_sample', 'Groupwise_Sampler', 'build_alias',
           'alias_draw', 'alias_distribution']
