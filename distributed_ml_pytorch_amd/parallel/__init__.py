"""Distributed runtime: flat arena, PS protocol, ASGD optimizer, sync DP."""
from .arena import FlatArena, attach_arena, get_arena
from .async_sharded import AsyncShardedPSClient, ShardServer
from .asgd import Asynchronous, DownpourSGD, default_client
from .clients import GlooPSClient, LocalPSClient, PSClient, RcclPSClient, ShardedPSClient
from .ddp import BucketedAllReduce, FusedSGD
from .messaging import MessageCode, MessageListener, SendTracker, send_message
from .server import ParameterServer, make_ps_groups

__all__ = ["FlatArena", "attach_arena", "get_arena", "Asynchronous", "DownpourSGD",
           "default_client", "GlooPSClient", "LocalPSClient", "PSClient", "RcclPSClient",
           "ShardedPSClient", "AsyncShardedPSClient", "ShardServer", "BucketedAllReduce", "FusedSGD", "MessageCode", "MessageListener",
           "SendTracker", "send_message", "ParameterServer", "make_ps_groups"]
