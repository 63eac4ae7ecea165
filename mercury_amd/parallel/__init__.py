"""Data-parallel runtime: process groups, flat buffers, bucketed RCCL all-reduce,
explicit ring all-reduce, importance-score all-gather."""
from .dist import (init_from_env, init_processes, spawn, free_port, rank, world_size,
                   is_initialized)
from .ring import allreduce
from .flat import FlatParams
from .buckets import BucketedAllReduce, default_bucket_bytes
from .scores import ScoreExchange

__all__ = ['init_from_env', 'init_processes', 'spawn', 'free_port', 'rank', 'world_size',
           'is_initialized', 'allreduce', 'FlatParams', 'BucketedAllReduce',
           'default_bucket_bytes', 'ScoreExchange']
