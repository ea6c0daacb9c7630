"""Model zoo for the flagship configs (GPT-3, BERT, ResNet via vision.models, LeNet)."""
from .gpt import (GPTConfig, GPTModel, GPTForPretraining, gpt_config, GPT_CONFIGS,  # noqa
                  gpt_flops_per_token)
from .bert import (BertConfig, BertModel, BertForPretraining, BertPretrainingCriterion,  # noqa
                   BertForSequenceClassification, BertForTokenClassification,
                   BertForQuestionAnswering, bert_config, BERT_CONFIGS, ErnieConfig, ErnieModel,
                   ErnieForPretraining, ErnieForSequenceClassification, ernie_config, ernie_pipe,
                   bert_flops_per_token)
