package jwave.hip;

import java.nio.ByteBuffer;
import java.nio.ByteOrder;
import java.util.concurrent.atomic.AtomicInteger;

import jwave.transforms.MODWTTransform;
import jwave.transforms.wavelets.Wavelet;

/**
 * Drop-in for {@link MODWTTransform}: forwardMODWT / inverseMODWT run on the MI355X through
 * jw_modwt_forward / jw_modwt_inverse (MODWTTransform.java:256-306, :337-375).  Callers keep
 * {@code new Transform(new HipMODWTTransform(w))}; the flattened forward/reverse API (:388-443,
 * :853-912) calls these overrides, so it needs no glue of its own.
 *
 * <p>With ARITH_STRICT (the default) every method is bit-identical to the JVM's: DIRECT, and
 * AUTO / FFT, which decide per level with the reference's int32 rule (N * M_j >
 * fftConvolutionThreshold takes the FFT path, :653) and run the reference's own FFT convolution
 * on the FFT levels (radix-2 with recurrence twiddles, Bluestein for other lengths, :752-837).
 * ARITH_FMA is the fast contract: AUTO runs DIRECT, FFT an exact-twiddle pyramid.
 * The plan (normalised filters, :452-484 and :599-606) is immutable and shared by all threads;
 * {@link #clearFilterCache()} retires it once no call holds it.
 */
public class HipMODWTTransform extends MODWTTransform {
  static {
    HipEngine.load();
  }

  public static final int ARITH_STRICT = 0, ARITH_FMA = 1;

  private final int arith;
  private final int device; // -1: the calling thread's current device
  private final Object planLock = new Object();
  private Plan plan; // guarded by planLock

  /** Reference-counted native plan: destroyed when retired and no call holds it. */
  private static final class Plan {
    final long handle;
    final AtomicInteger users = new AtomicInteger(1); // 1 = the transform's own reference

    Plan(long h) { handle = h; }

    void release() {
      if (users.decrementAndGet() == 0) nPlanDestroy(handle);
    }
  }

  /** MODWTTransform(wavelet) (:180-183): threshold 4096 (:144), AUTO (:167), STRICT. */
  public HipMODWTTransform(Wavelet w) {
    super(w);
    this.arith = ARITH_STRICT;
    this.device = -1;
  }

  /**
   * MODWTTransform(wavelet, fftThreshold) (:191-194), STRICT.  The second int is the threshold,
   * as in the reference, so {@code new HipMODWTTransform(w, 8192)} means what it means there;
   * the arithmetic contract takes the three-argument form.
   */
  public HipMODWTTransform(Wavelet w, int fftThreshold) { this(w, fftThreshold, ARITH_STRICT, -1); }

  public HipMODWTTransform(Wavelet w, int fftThreshold, int arith) { this(w, fftThreshold, arith, -1); }

  /** On GPU {@code device} (jw_set_device before every native call of the calling thread). */
  public HipMODWTTransform(Wavelet w, int fftThreshold, int arith, int device) {
    super(w, fftThreshold); // MODWTTransform.java:191
    this.arith = arith;
    this.device = device;
  }

  private Plan acquire() {
    if (device >= 0) HipEngine.setDevice(device);
    synchronized (planLock) {
      if (plan == null) {
        Wavelet w = getWavelet();
        plan = new Plan(nPlanCreate(w.getScalingDeComposition(), w.getWaveletDeComposition(),
                                    fftConvolutionThreshold, arith)); // protected field, :144
      }
      plan.users.incrementAndGet();
      return plan;
    }
  }

  @Override
  public double[][] forwardMODWT(double[] data, int maxLevel) {
    Plan p = acquire();
    try {
      return nForward(p.handle, data, maxLevel, getConvolutionMethod().ordinal());
    } finally {
      p.release();
    }
  }

  @Override
  public double[] inverseMODWT(double[][] coefficients) {
    if (coefficients == null || coefficients.length == 0 || coefficients[0].length == 0)
      return new double[0]; // MODWTTransform.java:338-346
    Plan p = acquire();
    try {
      return nInverse(p.handle, coefficients, getConvolutionMethod().ordinal());
    } finally {
      p.release();
    }
  }

  /**
   * Batched forward over direct buffers (native order): x holds batch signals of n samples,
   * coeffs receives batch x (maxLevel+1) x n.  One JNI crossing and one HBM staging for the
   * whole batch.
   */
  public void forwardMODWT(ByteBuffer x, ByteBuffer coeffs, int n, int maxLevel, int batch) {
    checkDirect(x, coeffs);
    Plan p = acquire();
    try {
      nForwardDirect(p.handle, x, coeffs, n, maxLevel, batch, getConvolutionMethod().ordinal());
    } finally {
      p.release();
    }
  }

  /** Batched inverse over direct buffers: coeffs batch x (levels+1) x n -> x batch x n. */
  public void inverseMODWT(ByteBuffer coeffs, ByteBuffer x, int n, int levels, int batch) {
    checkDirect(coeffs, x);
    Plan p = acquire();
    try {
      nInverseDirect(p.handle, coeffs, x, n, levels, batch, getConvolutionMethod().ordinal());
    } finally {
      p.release();
    }
  }

  /** The engine reads direct buffers from their base address in native byte order. */
  private static void checkDirect(ByteBuffer a, ByteBuffer b) {
    for (ByteBuffer buf : new ByteBuffer[] {a, b}) {
      if (!buf.isDirect() || buf.position() != 0 || buf.order() != ByteOrder.nativeOrder())
        throw new IllegalArgumentException(
            "direct ByteBuffers at position 0 in native byte order required");
    }
  }

  @Override
  public void clearFilterCache() {
    super.clearFilterCache();
    synchronized (planLock) {
      if (plan != null) {
        plan.release(); // freed now, or by the last in-flight call
        plan = null;
      }
    }
    // Per instance, as in the reference (MODWTTransform.java:556): only this object's plan is
    // retired.  The process-wide device tables (twiddles, filter spectra, which are shared by
    // every transform with the same taps and length) are freed only by an explicit
    // HipEngine.releaseCaches(), which waits for every device and stalls other threads.
  }

  private static native long nPlanCreate(double[] scalDec, double[] wavDec, int fftThreshold,
                                         int arith);
  private static native void nPlanDestroy(long plan);
  private static native double[][] nForward(long plan, double[] x, int levels, int method);
  private static native double[] nInverse(long plan, double[][] c, int method);
  private static native void nForwardDirect(long plan, ByteBuffer x, ByteBuffer c, long n,
                                            int levels, int batch, int method);
  private static native void nInverseDirect(long plan, ByteBuffer c, ByteBuffer x, long n,
                                            int levels, int batch, int method);
}
