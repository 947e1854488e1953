"""Decode an image texture the reference loads through the `image` crate (ImageTexture::new,
texture.rs:302-318: image::open(..).to_rgb8()) into a binary PPM the C++ host reads.

    python tools/decode_image.py /root/reference/input/earthmap.jpg assets/earthmap.ppm

This container has Pillow (libjpeg-turbo); the reference's `image` 0.25 decodes JPEG with its own
decoder, so texel values may differ by an LSB here and there: texel parity with the reference is
unpinned. GPU and oracle read the same decoded texels, so their parity is bitwise."""
import sys

from PIL import Image


def main():
    src, dst = sys.argv[1], sys.argv[2]
    img = Image.open(src).convert("RGB")
    w, h = img.size
    with open(dst, "wb") as f:
        f.write(f"P6\n{w} {h}\n255\n".encode())
        f.write(img.tobytes())
    print(f"{src}: {w}x{h} -> {dst}")


if __name__ == "__main__":
    main()
