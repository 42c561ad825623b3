"""MI355X-native distributed exact k-NN classification framework.

Capabilities of jiajunchang2002g/Distributed-Machine-Learning-Project (a C++/MPI k-NN engine),
re-designed for AMD Instinct MI355X (gfx950): hand-written HIP/CDNA4 kernels for the hot loops,
RCCL over xGMI (torch.distributed "nccl" backend) for the data plane, C++ for the host runtime.

    import distributed_machine_learning_project_amd as dmlp
"""
__version__ = "0.1.0"

from .utils.io import (KNNInput, Params, DataPoint, Query, Update, parse_update,  # noqa: F401
                       parse_input, read_input, generate, generate_text, format_report, format_debug, to_text)
