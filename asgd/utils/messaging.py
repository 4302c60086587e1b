from distributed_ml_pytorch_amd.parallel.messaging import (  # noqa: F401
    MessageCode, MessageListener, SendTracker, recv_header, send_message)
