"""snake_amd — MI355X-native hot path of lucagiorgetti/Laplace-DQN-Snake-game.

Import as `import snake_amd` (the root shim snake_amd.py maps this hyphenated
directory to that name). All compute runs in libsnakehip.so (HIP, gfx950);
this package is the host-side mirror of the reference's Julia API.
"""
from ._lib import (BufferSizeError, DeviceArray, FoodListExhausted, SnakeHipError,  # noqa: F401
                   arith, device_count, get_arith, header_symbols, load, set_arith)
from .env import (ALL_ACTIONS, D, L, NULL_ACTION, R, U, SnakeGame, assemble_state_,  # noqa: F401
                  available_action_codes, available_actions, food_list, reset_, step_,
                  step_indices_dev, synth_actions_dev, virtual_step)
from .replay import (ReplayBuffer, empty_buffer_, isfull, isready, sample, stack_exp,  # noqa: F401
                     store_)
from ._lib import SNK_NET_GRAD, SNK_NET_OPT_STATE, SNK_NET_Q, SNK_NET_TARGET  # noqa: F401
from .qnet import DQNModel, deep_nparams, nparams, update_target_net_  # noqa: F401
from .dist import Comm, aggregate_throughput, dist_attach, dist_detach  # noqa: F401
from .trainer import Trainer, epsilon_greedy, fill_buffer_, play_episode, train_  # noqa: F401
from .laplace import (LaplaceD, compute_D, gram_tiles, jacobian, jacobian_gram,  # noqa: F401
                      jacobian_gram_gather, jacobian_gram_shard, laplace_normals, laplace_sampling_,
                      sample_model)
from .bsonio import load_trainer, read_trainer  # noqa: F401
from . import gif  # noqa: F401

__version__ = "1.0.0"
