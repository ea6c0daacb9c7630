"""Model zoo for the flagship configs (GPT-3, BERT, ResNet via vision.models, LeNet)."""
from .gpt import (GPTConfig, GPTModel, GPTForPretraining, gpt_config, GPT_CONFIGS,  # noqa
                  gpt_flops_per_token)
