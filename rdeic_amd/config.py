"""Model configuration of the RDEIC hot path (mirrors configs/model/rdeic.yaml of the reference:
unet_config :54-70, control_stage_config :33-52, first_stage_config :72-94, preprocess_config
:102-111, schedule :2-4,15,26). Keys keep the reference's constructor argument names."""
import copy

_UNET = dict(image_size=32, in_channels=4, out_channels=4, model_channels=320, attention_resolutions=[4, 2, 1],
             num_res_blocks=2, channel_mult=[1, 2, 4, 4], num_head_channels=64, use_spatial_transformer=True,
             use_linear_in_transformer=True, transformer_depth=1, context_dim=1024, legacy=False,
             use_checkpoint=False)

CONFIG = dict(
    unet=_UNET,
    control=dict(_UNET, hint_channels=256, num_head_channels=16, control_model_ratio=0.2, control_scale=1.0),
    ddconfig=dict(double_z=True, z_channels=4, resolution=256, in_channels=3, out_ch=3, ch=128,
                  ch_mult=[1, 2, 4, 4], num_res_blocks=2, attn_resolutions=[], dropout=0.0),
    embed_dim=4,
    compression=dict(in_nc=512, out_nc=4, N=256, M=256, slice_num=10, slice_ch=[8, 8, 8, 8, 16, 16, 32, 32, 64, 64],
                     codebook_size=16384),
    scale_factor=0.18215,
    linear_start=0.00085,
    linear_end=0.0120,
    timesteps=1000,
    used_timesteps=300,
    context_len=77,
)


def default_config():
    return copy.deepcopy(CONFIG)
