package jwave.hip;

import jwave.datatypes.natives.Complex;
import jwave.transforms.CWTResult;
import jwave.transforms.ContinuousWaveletTransform;
import jwave.transforms.wavelets.continuous.ContinuousWavelet;
import jwave.transforms.wavelets.continuous.DOGWavelet;
import jwave.transforms.wavelets.continuous.MeyerWavelet;
import jwave.transforms.wavelets.continuous.MexicanHatWavelet;
import jwave.transforms.wavelets.continuous.MorletWavelet;
import jwave.transforms.wavelets.continuous.PaulWavelet;

/**
 * Drop-in for {@link ContinuousWaveletTransform}: transformFFT / transformFFTParallel
 * (ContinuousWaveletTransform.java:183-229, :511-565) through jw_cwt_fft, and the direct
 * transform / transformParallel (:141-172, :470-500) through jw_cwt_direct.  Wavelets the
 * engine does not know fall back to the reference implementation (super).
 */
public class HipContinuousWaveletTransform extends ContinuousWaveletTransform {
  static {
    HipEngine.load();
  }

  private final ContinuousWavelet wavelet;
  private final int padding; // PaddingType.ordinal(): the reference keeps it private (:84)
  private final int arith;
  private final int device; // -1: the calling thread's current device

  /** The reference's default padding is SYMMETRIC (ContinuousWaveletTransform.java:91-93). */
  public HipContinuousWaveletTransform(ContinuousWavelet w) {
    this(w, PaddingType.SYMMETRIC, HipMODWTTransform.ARITH_STRICT);
  }

  /** ContinuousWaveletTransform(wavelet, paddingType) (:101-106), STRICT arithmetic. */
  public HipContinuousWaveletTransform(ContinuousWavelet w, PaddingType p) {
    this(w, p, HipMODWTTransform.ARITH_STRICT);
  }

  public HipContinuousWaveletTransform(ContinuousWavelet w, PaddingType p, int arith) {
    this(w, p, arith, -1);
  }

  /** On GPU {@code device} (jw_set_device before every native call of the calling thread). */
  public HipContinuousWaveletTransform(ContinuousWavelet w, PaddingType p, int arith, int device) {
    super(w, p);
    wavelet = w;
    padding = p.ordinal();
    this.arith = arith;
    this.device = device;
  }

  private void onDevice() {
    if (device >= 0) HipEngine.setDevice(device);
  }

  /** JW_CWT_* kind, or -1 when the engine has no kernel for this wavelet class. */
  private int kind() {
    if (wavelet instanceof MorletWavelet) return 0;
    if (wavelet instanceof MexicanHatWavelet) return 1;
    if (wavelet instanceof PaulWavelet) return 2;
    if (wavelet instanceof DOGWavelet) return 3;
    if (wavelet instanceof MeyerWavelet) return 4;
    return -1;
  }

  private double[] params() {
    if (wavelet instanceof MorletWavelet) {
      MorletWavelet m = (MorletWavelet) wavelet;
      return new double[] {m.getBandwidthParameter(), m.getCenterFrequencyParameter()};
    }
    if (wavelet instanceof MexicanHatWavelet)
      return new double[] {((MexicanHatWavelet) wavelet).getSigma()};
    if (wavelet instanceof PaulWavelet) return new double[] {((PaulWavelet) wavelet).getOrder()};
    if (wavelet instanceof DOGWavelet) {
      DOGWavelet d = (DOGWavelet) wavelet;
      return new double[] {d.getDerivativeOrder(), d.getSigma()};
    }
    return new double[0];
  }

  private CWTResult result(double[][] rows, double[] scales, int n, double fs) {
    Complex[][] c = new Complex[rows.length][n];
    for (int s = 0; s < rows.length; s++)
      for (int t = 0; t < n; t++) c[s][t] = new Complex(rows[s][2 * t], rows[s][2 * t + 1]);
    double[] time = new double[n];
    double dt = 1.0 / fs; // createTimeAxis, :423-430
    for (int i = 0; i < n; i++) time[i] = i * dt;
    return new CWTResult(c, scales, time, fs, wavelet.getName());
  }

  @Override
  public CWTResult transformFFT(double[] signal, double[] scales, double samplingRate) {
    int k = kind();
    if (k < 0) return super.transformFFT(signal, scales, samplingRate);
    onDevice();
    double[][] rows = nTransformFFT(k, params(), signal, scales, samplingRate, padding);
    return result(rows, scales, signal.length, samplingRate);
  }

  /**
   * transformFFT(signal, scales, samplingRate).getScalogram() (CWTResult.java:272-287) with the
   * ns x n coefficients kept on the GPU: only the ns energies cross PCIe.
   */
  public double[] transformFFTScalogram(double[] signal, double[] scales, double samplingRate) {
    int k = kind();
    if (k < 0) return super.transformFFT(signal, scales, samplingRate).getScalogram();
    onDevice();
    return nScalogramFFT(k, params(), signal, scales, samplingRate, padding);
  }

  @Override
  public CWTResult transformFFTParallel(double[] signal, double[] scales, double samplingRate) {
    return transformFFT(signal, scales, samplingRate); // same values (:511-565)
  }

  @Override
  public CWTResult transform(double[] signal, double[] scales, double samplingRate) {
    int k = kind();
    if (k < 0) return super.transform(signal, scales, samplingRate);
    onDevice();
    double[][] rows = nTransformDirect(k, params(), signal, scales, samplingRate, arith);
    return result(rows, scales, signal.length, samplingRate);
  }

  @Override
  public CWTResult transformParallel(double[] signal, double[] scales, double samplingRate) {
    return transform(signal, scales, samplingRate); // same values (:470-500)
  }

  /**
   * transformParallelCustom (ContinuousWaveletTransform.java:577-680) computes the same values
   * as transform with a caller-sized ForkJoinPool; on the GPU the pool size has no meaning.
   */
  @Override
  public CWTResult transformParallelCustom(double[] signal, double[] scales, double samplingRate,
                                           int parallelism) {
    if (kind() < 0)
      return super.transformParallelCustom(signal, scales, samplingRate, parallelism);
    return transform(signal, scales, samplingRate);
  }

  private static native double[][] nTransformFFT(int kind, double[] params, double[] x,
                                                 double[] scales, double fs, int padding);
  private static native double[] nScalogramFFT(int kind, double[] params, double[] x,
                                               double[] scales, double fs, int padding);
  private static native double[][] nTransformDirect(int kind, double[] params, double[] x,
                                                    double[] scales, double fs, int arith);
}
