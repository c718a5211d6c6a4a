"""Encoder factory (mirror of reference encoding.py:5-33)."""


def get_encoder(encoding, input_dim=3, multires=6, degree=4, num_levels=16, level_dim=2,
                base_resolution=16, log2_hashmap_size=19, desired_resolution=2048,
                align_corners=False, **kwargs):
    """Return (encoder module, output dim) for one of
    None / frequency / sphere_harmonics / hashgrid / tiledgrid."""
    if encoding == "None":
        return (lambda x, **kw: x), input_dim
    if encoding == "frequency":
        from freqencoder import FreqEncoder
        enc = FreqEncoder(input_dim=input_dim, degree=multires)
    elif encoding == "sphere_harmonics":
        from shencoder import SHEncoder
        enc = SHEncoder(input_dim=input_dim, degree=degree)
    elif encoding in ("hashgrid", "tiledgrid"):
        from gridencoder import GridEncoder
        enc = GridEncoder(input_dim=input_dim, num_levels=num_levels, level_dim=level_dim,
                          base_resolution=base_resolution, log2_hashmap_size=log2_hashmap_size,
                          desired_resolution=desired_resolution,
                          gridtype="hash" if encoding == "hashgrid" else "tiled",
                          align_corners=align_corners)
    else:
        raise NotImplementedError("Unknown encoding mode, choose from "
                                  "[None, frequency, sphere_harmonics, hashgrid, tiledgrid]")
    return enc, enc.output_dim
