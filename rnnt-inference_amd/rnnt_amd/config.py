"""Model constants of the MLPerf RNN-T.

Mirrors ``RNNTParam`` (reference ``models/config.py:1-19``) and the C++ ``Params`` enum
(``csrc/metadata.hpp:19-34``), plus the engine's padded sizes.
"""


class RNNTParam:
    # Transcription (encoder)
    trans_input_size = 240  # 80 mel x 3 spliced frames
    trans_hidden_size = 1024
    pre_num_layers = 2
    post_num_layers = 3
    stack_time_factor = 2
    # Prediction
    pred_hidden_size = 320
    pred_num_layers = 2
    # Joint
    joint_hidden_size = 512
    num_labels = 29
    # [SOS, SPACE, a~z, ', BLANK] = [-1, 0, 1~26, 27, 28]
    SOS = -1
    BLANK = 28
    max_symbols_per_step = 30
    sample_rate = 16000
    # csrc/metadata.hpp:31-33
    MAX_WAV_LEN = 240000
    MAX_FEA_LEN = 500
    PADDED_INPUT_SIZE = 256


# Encoder layer input widths after padding (layer 0: 240 -> 256 zero-padded channels,
# reference quant_lstm.py:235-236 / metadata.hpp:33) and the stacked post_rnn input.
ENC_INPUT_SIZES = (256, 1024, 2048, 1024, 1024)
ENC_K = tuple(i + RNNTParam.trans_hidden_size for i in ENC_INPUT_SIZES)  # 1280,2048,3072,2048,2048
NUM_ENC_LAYERS = 5
LABELS_PADDED = 32  # joint linear2 output padded 29 -> 32 (modeling_rnnt.py:241-250)

# labels, reference models/utils.py:23-52 and csrc/metadata.hpp:15-17
LABELS = [" "] + [chr(ord("a") + i) for i in range(26)] + ["'"]


def seq_to_sen(seq, seq_len):
    """reference models/utils.py:55-57"""
    return "".join(LABELS[int(seq[i])] for i in range(int(seq_len)))


def encoder_frames(feature_len):
    """f_lens = ceil(x_lens / stack_time_factor) (decoder.py:185, rnnt_model.hpp:88-89)."""
    return (int(feature_len) + RNNTParam.stack_time_factor - 1) // RNNTParam.stack_time_factor


def encoder_ops(T):
    """Algorithmic int8 ops of one utterance of T valid feature frames:
    2*4H*[(240+H) + 2H]*T + 2*4H*[(2H+H) + 2H + 2H]*ceil(T/2)."""
    H = RNNTParam.trans_hidden_size
    return 2 * 4 * H * ((240 + H) + 2 * H) * T + 2 * 4 * H * (3 * H + 2 * H + 2 * H) * encoder_frames(T)
