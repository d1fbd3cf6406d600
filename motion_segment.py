"""Drop-in for the reference CLI ``motion_segment.py`` (flags :19-65, outputs :117-150) on the
MI355X engine: segment and motion-track the LV in an echo video, print EF, write pickles.

Same flags and defaults. ``-d/--device`` keeps the reference default ``cpu``. In the reference that
runs the model on the host CPU; this engine has no CPU compute path, so -- a deliberate extension,
announced by a notice -- ``-d cpu`` runs the engine on GPU 0 and returns host arrays, exactly as
``-d cuda`` does (the outputs are numpy int64 arrays either way). Without a GPU the CLI exits with
an error. ``-d cuda`` / ``cuda:i`` pick the GPU.
Extra opt-in flags: ``--synthetic-weights SEED`` with ``--synthetic-recipe echo|random`` (seeded
weights when no checkpoint is available offline), ``--batch-size`` (clips per forward call) and
``--no-strict-reference`` (fuse_utils.segment_a_video_with_fusion(strict_reference=False)).
Video input: any file OpenCV can decode if cv2 is installed (as the reference), or ``.npy`` holding
(T,H,W,3) uint8 RGB frames.
"""
import argparse
import os
import pickle
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))


def parse_args(argv=None):
    ap = argparse.ArgumentParser(description="Segment and motion track heart structure in an Echo Video")
    ap.add_argument("-p", "--path", required=True, type=str, help="Path to the video")
    ap.add_argument("-m", "--model", required=False, type=str, help="Path to the saved model weights",
                    default="save_models/R2plus1DMotionSegNet_model.pth")
    ap.add_argument("-d", "--device", required=False, type=str, help="Which device to use: CPU or GPU",
                    default="cpu")
    ap.add_argument("--fuse_method", required=False, type=str, help="Fuse method", default="simple")
    ap.add_argument("-f", "--fuse", required=False, type=int, help="Number of shifted video clips to fuse", default=1)
    ap.add_argument("-s", "--step", required=False, type=int, help="Step of shifting", default=1)
    ap.add_argument("-o", "--output", required=False, type=str, help="Path to the output files", default=".")
    ap.add_argument("-v", "--verbose", action="store_true", help="Verbosity")
    ap.add_argument("-c", "--content", required=False, type=str,
                    help="Content of the output: gif, binary, binary_video, all", default="binary")
    ap.add_argument("--height", required=False, type=int, help="Height of image (pretrain model uses 112)", default=112)
    ap.add_argument("--width", required=False, type=int, help="Width of image (pretrain model uses 112)", default=112)
    ap.add_argument("--synthetic-weights", type=int, default=None, metavar="SEED",
                    help="use seeded synthetic weights instead of a checkpoint (no trained weights offline)")
    ap.add_argument("--synthetic-recipe", choices=["echo", "random"], default="echo",
                    help="synthetic weight recipe: 'echo' segments the LV of EchoNet-style videos (physiological "
                         "EFs), 'random' is plain seeded noise")
    ap.add_argument("--batch-size", type=int, default=32, help="clips per forward call")
    ap.add_argument("--no-strict-reference", action="store_true",
                    help="correct the reference's plumbing quirks: a single 32-frame clip yields masks instead of "
                         "IndexError, and frames 1..step-1 are kept for step > 1")
    return ap.parse_args(argv)


def read_video(path):
    """(T,H,W,3) uint8 RGB, as motion_segment.py:80-94."""
    if path.endswith(".npy"):
        v = np.load(path, allow_pickle=False)
        if v.ndim != 4 or v.shape[-1] != 3:
            raise ValueError(f"{path}: expected (T,H,W,3) frames, got {v.shape}")
        return v.astype(np.uint8)
    try:
        import cv2
    except ImportError as e:
        raise RuntimeError(f"{path}: OpenCV (cv2) is not installed; provide frames as a .npy file") from e
    cap = cv2.VideoCapture(path)
    n, w, h = (int(cap.get(cv2.CAP_PROP_FRAME_COUNT)), int(cap.get(cv2.CAP_PROP_FRAME_WIDTH)),
               int(cap.get(cv2.CAP_PROP_FRAME_HEIGHT)))
    video = np.zeros((n, h, w, 3), np.uint8)
    for i in range(n):
        ok, frame = cap.read()
        if not ok:
            raise ValueError("Failed to load frame #{} of {}.".format(i, path))
        video[i] = cv2.cvtColor(frame, cv2.COLOR_BGR2RGB)
    return video


def main(argv=None):
    args = parse_args(argv)
    host_io = args.device.lower().startswith("cpu")
    if not torch.cuda.is_available():
        sys.exit("error: the CLAS-FV engine needs an MI355X (ROCm) GPU and none is visible")
    if host_io:
        print("notice: -d cpu: this engine has no CPU compute path; the engine runs on GPU 0 and the outputs "
              "are host arrays", file=sys.stderr)
        dev = torch.device("cuda", 0)
    else:
        dev = torch.device(args.device)
        if dev.type != "cuda":
            sys.exit(f"error: unknown device {args.device!r}; use cpu, cuda or cuda:i")
        if dev.index is None:
            dev = torch.device("cuda", torch.cuda.current_device())
    torch.cuda.set_device(dev)

    from clasfv_amd.echo import compute_ef_using_putative_clips
    from clasfv_amd.fuse_utils import segment_a_video_with_fusion
    from clasfv_amd.model import R2plus1D_18_MotionNet
    from clasfv_amd.preprocess import preprocess_video
    from clasfv_amd.weights import DEFAULT_SEED, load_checkpoint

    seed = args.synthetic_weights if args.synthetic_weights is not None else DEFAULT_SEED
    model = R2plus1D_18_MotionNet(pretrained=False, seed=seed, device=dev, weights=args.synthetic_recipe)
    if args.synthetic_weights is None:
        model.load_state_dict(load_checkpoint(args.model))
    if args.verbose:
        print(f"R2+1D MotionNet has {sum(p.numel() for p in model.parameters() if p.requires_grad)} parameters.")
    model.eval()

    # motion_segment.py:96-106 on the device: uint8 frames -> resize -> zero-one normalisation
    video = preprocess_video(read_video(args.path), args.height, args.width, device=dev)

    segmentations = segment_a_video_with_fusion(video, model=model, interpolate_last=True, step=args.step,
                                                num_clips=args.fuse, fuse_method=args.fuse_method, class_list=[0, 1],
                                                batch_size=args.batch_size,
                                                strict_reference=not args.no_strict_reference)
    predicted_efs, edes_pairs = compute_ef_using_putative_clips(segmentations, test_pat_index=args.path,
                                                                return_edes=True)
    if args.verbose:
        print("Identified {:d} systoles".format(len(predicted_efs)))
        if len(predicted_efs) > 0:
            print("\nEjection fractions measured at each systole are:")
            for i in range(len(predicted_efs)):
                print("Systole #{:d}: ED {:d} & ES {:d} length={:d}".format(
                    i + 1, edes_pairs[i][0], edes_pairs[i][1], edes_pairs[i][1] - edes_pairs[i][0]))
                print("EF: {:.2f}\n".format(predicted_efs[i]))
            print("The average ejection fraction is {:.2f}".format(np.mean(predicted_efs)))

    filename = args.path[args.path.rfind("/") + 1:args.path.rfind(".")]
    content = args.content.lower().split(",")
    if "gif" in content or "all" in content:
        print("warning: annotated GIF output (src/visualization_utils.py:476-539) is not part of this engine; skipped",
              file=sys.stderr)
    if "binary" in content or "all" in content:
        for ed_index, es_index in edes_pairs:
            with open(os.path.join(args.output, filename + "_ED_Frame_{:d}_segmentation.pkl".format(ed_index)), "wb") as f:
                pickle.dump(segmentations[ed_index], f)
            with open(os.path.join(args.output, filename + "_ES_Frame_{:d}_segmentation.pkl".format(es_index)), "wb") as f:
                pickle.dump(segmentations[es_index], f)
    if "binary_video" in content or "all" in content:
        with open(os.path.join(args.output, filename + "_whole_video_segmentation.pkl"), "wb") as f:
            pickle.dump(segmentations, f)
    return segmentations, predicted_efs, edes_pairs


if __name__ == "__main__":
    main()
