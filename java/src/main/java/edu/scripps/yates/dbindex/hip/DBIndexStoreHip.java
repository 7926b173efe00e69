package edu.scripps.yates.dbindex.hip;

import java.util.ArrayList;
import java.util.Iterator;
import java.util.List;

import edu.scripps.yates.dbindex.DBIndexStore;
import edu.scripps.yates.dbindex.ProteinCache;
import edu.scripps.yates.dbindex.Util;
import edu.scripps.yates.utilities.fasta.dbindex.DBIndexSearchParams;
import edu.scripps.yates.utilities.fasta.dbindex.DBIndexStoreException;
import edu.scripps.yates.utilities.fasta.dbindex.IndexedProtein;
import edu.scripps.yates.utilities.fasta.dbindex.IndexedSequence;
import edu.scripps.yates.utilities.fasta.dbindex.MassRange;
import edu.scripps.yates.utilities.fasta.dbindex.ResidueInfo;
import edu.scripps.yates.utilities.masses.AssignMass;

/**
 * {@link DBIndexStore} (DBIndexStore.java:19-194) on the MI355X engine: every
 * method is one call into libdbindex_hip.so through libdbindex_jni.so
 * (src/main/c/dbindex_jni.c), one {@code dbi_store_*} function of
 * include/dbindex_hip.h per method.  Injected through
 * {@code DBIndexer(sparam, mode, store)} (DBIndexer.java:143-155).
 *
 * With {@link #setDeviceDigest(boolean)} on (what {@link DBIndexerHip} does),
 * {@code addProteinDef} only collects the proteome and {@code stopAddSeq}
 * digests, sorts and de-duplicates it on the GPU; with it off, the store
 * indexes exactly the occurrences the stock {@code cutSeq} passes to
 * {@code addSequence}, like DBIndexStoreSQLiteMult.  A non-zero native status
 * is thrown as {@link DBIndexStoreException} with the library's message;
 * nothing is swallowed.
 */
public class DBIndexStoreHip implements DBIndexStore {
    static {
        System.loadLibrary("dbindex_jni");  // links libdbindex_hip.so
    }

    /** A List&lt;IndexedSequence&gt; in flat arrays (dbi_seq_list), filled by the native side. */
    static final class SeqList {
        double[] mass;
        int[] seqOff;      // n + 1
        byte[] seqChars;
        byte[] left;       // 3 per sequence (Util.getResidues, Util.java:130-162)
        byte[] right;
        int[] protOff;     // n + 1
        int[] protIds;
        int[] pepOff;      // first occurrence's offset in protein protIds[protOff[i]]
    }

    protected long h;  // dbi_store*
    private ProteinCache proteinCache;
    private int unindexedMode;     // dbi_store_set_unindexed mode (0: indexed store)
    private boolean cacheLoaded;   // unindexed: cache proteins handed to the device

    public DBIndexStoreHip(DBIndexSearchParams p, int device) throws DBIndexStoreException {
        final char[] mand = p.getMandatoryInternalAAs();
        h = create(massTable(), p.getEnzymeResidues(), p.getEnzymeNocutResidues(),
                mand == null ? null : new String(mand), p.getMaxMissedCleavages(), p.isSemiCleavage(),
                p.getMinPrecursorMass(), p.getMaxPrecursorMass(), p.isH2OPlusProtonAdded(),
                AssignMass.H2O_PROTON, AssignMass.getcTerm(), AssignMass.getnTerm(), p.getMassGroupFactor(),
                p.getIndexFactor(), device);
    }

    /**
     * AssignMass.getMass(c) for every char (DBIndexer.java:306): the engine sums
     * the caller's own table, so static modifications the params file added
     * (SearchParamReader.java:401-583) are in it.
     */
    private static double[] massTable() {
        final double[] t = new double[256];
        for (int c = 0; c < 256; c++) {
            t[c] = AssignMass.getMass((char) c);
        }
        return t;
    }

    // ---- DBIndexStore ------------------------------------------------------------
    @Override
    public void init(String databaseID) throws DBIndexStoreException {          // :37
        init0(h, databaseID);
    }

    @Override
    public void startAddSeq() throws DBIndexStoreException {                    // :45
        startAddSeq0(h);
    }

    @Override
    public void stopAddSeq() throws DBIndexStoreException {                     // :54 (the GPU build)
        stopAddSeq0(h);
    }

    @Override
    public boolean indexExists() throws DBIndexStoreException {                 // :61
        return indexExists0(h);
    }

    @Override
    public FilterResult filterSequence(double precMass, String sequence) {      // :74
        switch (filterSequence0(h, precMass, sequence)) {
        case 0:
            return FilterResult.INCLUDE;
        case 1:
            return FilterResult.SKIP;
        default:
            return FilterResult.SKIP_PROTEIN_START;
        }
    }

    @Override
    public void addSequence(double precMass, int sequenceOffset, int sequenceLen, String sequence,
            String resLeft, String resRight, long proteinId) throws DBIndexStoreException {  // :96
        addSequence0(h, precMass, sequenceOffset, sequenceLen, proteinId);
    }

    @Override
    public List<IndexedSequence> getSequences(double precMass, double tolerance)
            throws DBIndexStoreException {                                      // :114
        return toList(getSequences0(h, precMass, tolerance));
    }

    @Override
    public List<IndexedSequence> getSequences(List<MassRange> ranges) throws DBIndexStoreException {  // :127
        final double[] m = new double[ranges.size()];
        final double[] t = new double[ranges.size()];
        for (int i = 0; i < m.length; i++) {
            m[i] = ranges.get(i).getPrecMass();
            t[i] = ranges.get(i).getTolerance();
        }
        return toList(getSequencesRanges0(h, m, t));
    }

    @Override
    public Iterator<IndexedSequence> getSequencesIterator(List<MassRange> ranges) throws DBIndexStoreException {
        return getSequences(ranges).iterator();
    }

    @Override
    public long addProteinDef(long num, String accession, String protSequence) throws DBIndexStoreException {
        return addProteinDef0(h, num, accession, protSequence);                // :144, returns num
    }

    @Override
    public void setProteinCache(ProteinCache protCache) {                      // :152
        proteinCache = protCache;
        if (unindexedMode != 0 && protCache != null && !cacheLoaded) {
            // SEARCH_UNINDEXED: DBIndexer.setProteinCache (:461-500) fills the cache
            // from the FASTA; its proteins go to the device once, where the
            // reference re-cuts them on every cutAndSearch (:707-747)
            try {
                startAddSeq0(h);
                for (int i = 0; i < protCache.getNumberProteins(); i++) {
                    addProteinDef0(h, i, protCache.getDef(i), protCache.getProteinSequence(i));
                }
                stopAddSeq0(h);
            } catch (final DBIndexStoreException e) {
                throw new RuntimeException(e);
            }
            cacheLoaded = true;
        }
    }

    /**
     * DBIndexer.cutAndSearch (DBIndexer.java:707-747) on the unindexed store: the
     * MassRangeFilteringIndex init + cutSeq of every cached protein + getSequences
     * in one device pass.  Errors propagate (the reference logs them and returns null).
     */
    public List<IndexedSequence> cutAndSearch(List<MassRange> ranges) throws DBIndexStoreException {
        final double[] m = new double[ranges.size()];
        final double[] t = new double[ranges.size()];
        for (int i = 0; i < m.length; i++) {
            m[i] = ranges.get(i).getPrecMass();
            t[i] = ranges.get(i).getTolerance();
        }
        return toList(cutAndSearch0(h, m, t));
    }

    @Override
    public boolean supportsProteinCache() {                                     // :159
        return true;
    }

    @Override
    public List<IndexedProtein> getProteins(IndexedSequence sequence) throws DBIndexStoreException {  // :171
        final List<IndexedProtein> ret = new ArrayList<IndexedProtein>();
        for (final Integer protId : sequence.getProteinIds()) {
            // the cache's definition when one is set (SQLiteMult.java:457)
            ret.add(new IndexedProtein(proteinCache != null ? proteinCache.getDef(protId) : proteinDef0(h, protId),
                    protId));
        }
        return ret;
    }

    @Override
    public long getNumberSequences() throws DBIndexStoreException {             // :180 (mass-key rows)
        return getNumberSequences0(h);
    }

    @Override
    public ResidueInfo getResidues(IndexedSequence peptideSequence, IndexedProtein protein)
            throws DBIndexStoreException {                                      // :190
        // as DBIndexStoreSQLiteMult.getResidues (:294-312): the peptide's own
        // offset, else its first position in the protein
        final String proteinSequence = proteinCache != null ? proteinCache.getProteinSequence(protein.getId())
                : proteinSequence0(h, protein.getId());
        int seqOffset = peptideSequence.getSequenceOffset();
        if (seqOffset == IndexedSequence.OFFSET_UNKNOWN) {
            seqOffset = proteinSequence.indexOf(peptideSequence.getSequence());
        }
        if (seqOffset == -1) {
            throw new DBIndexStoreException("peptide " + peptideSequence.getSequence() + " is not in protein "
                    + protein.getId());
        }
        return Util.getResidues(peptideSequence, seqOffset, peptideSequence.getSequenceLen(), proteinSequence);
    }

    @Override
    public List<Integer> getEntryKeys() throws DBIndexStoreException {          // :192
        final int[] k = getEntryKeys0(h);
        final List<Integer> ret = new ArrayList<Integer>(k.length);
        for (final int x : k) {
            ret.add(x);
        }
        return ret;
    }

    @Override
    public void lastBuffertoDatabase() {
        // no write buffer: the index lives in HBM
    }

    /** DBIndexerHip's hook: the GPU digests the proteome at stopAddSeq (dbi_store_set_device_digest). */
    public void setDeviceDigest(boolean on) throws DBIndexStoreException {
        setDeviceDigest0(h, on);
    }

    /** indexExists() reuse across processes (dbi_store_set_persist; DBIndexer.java:522-527). */
    public void setPersist(boolean on) throws DBIndexStoreException {
        setPersist0(h, on);
    }

    /** SEARCH_UNINDEXED store (dbi_store_set_unindexed: 1 resident, 2 stream), before init. */
    public void setUnindexed(int mode) throws DBIndexStoreException {
        setUnindexed0(h, mode);
        unindexedMode = mode;
    }

    /** Total occurrences indexed (DBIndexStoreSQLiteMult.totalSeqCount, :277). */
    public long getTotalSeqCount() throws DBIndexStoreException {
        return getTotalSeqCount0(h);
    }

    public void close() {
        if (h != 0) {
            close0(h);
            h = 0;
        }
    }

    /**
     * IndexMerge.parseAddPeptideInfo (:446-470): sequence, mass, protein ids,
     * flanks.  With a ProteinCache set, text and flanks come from the cache
     * entry of the first protein id, as the reference stores do
     * (IndexMerge.java:452-461): that differs from the store's own copy only
     * when DBIndexer.run discarded decoys ahead of targets (the cache holds
     * every protein, DBIndexer.java:605; ids count non-decoys, :609-616), and
     * the reference's shifted answers are then reproduced.
     */
    List<IndexedSequence> toList(SeqList l) {
        final int n = l.mass.length;
        final List<IndexedSequence> ret = new ArrayList<IndexedSequence>(n);
        for (int i = 0; i < n; i++) {
            final int len = l.seqOff[i + 1] - l.seqOff[i];
            final int pid0 = l.protIds[l.protOff[i]];
            String seq;
            ResidueInfo res;
            if (proteinCache != null) {
                seq = proteinCache.getPeptideSequence(pid0, l.pepOff[i], len);
                res = Util.getResidues(null, l.pepOff[i], len, proteinCache.getProteinSequence(pid0));
            } else {
                seq = new String(l.seqChars, l.seqOff[i], len, java.nio.charset.StandardCharsets.ISO_8859_1);
                res = new ResidueInfo(new String(l.left, 3 * i, 3, java.nio.charset.StandardCharsets.ISO_8859_1),
                        new String(l.right, 3 * i, 3, java.nio.charset.StandardCharsets.ISO_8859_1));
            }
            final IndexedSequence s = new IndexedSequence(0, l.mass[i], seq, "", "");
            final List<Integer> ids = new ArrayList<Integer>(l.protOff[i + 1] - l.protOff[i]);
            for (int k = l.protOff[i]; k < l.protOff[i + 1]; k++) {
                ids.add(l.protIds[k]);
            }
            s.setProteinIds(ids);
            s.setResidues(res);
            ret.add(s);
        }
        return ret;
    }

    // ---- natives (src/main/c/dbindex_jni.c) -----------------------------------------
    private static native long create(double[] mass, String cleave, String nocut, String mandatory,
            int maxMissed, boolean semi, double minMH, double maxMH, boolean addH2O, double h2oProton,
            double cTerm, double nTerm, int massGroupFactor, int indexFactor, int device)
            throws DBIndexStoreException;

    private static native void close0(long h);

    private static native void init0(long h, String databaseID) throws DBIndexStoreException;

    private static native void startAddSeq0(long h) throws DBIndexStoreException;

    private static native void stopAddSeq0(long h) throws DBIndexStoreException;

    private static native boolean indexExists0(long h) throws DBIndexStoreException;

    private static native int filterSequence0(long h, double mass, String sequence);

    private static native void addSequence0(long h, double mass, int offset, int length, long proteinId)
            throws DBIndexStoreException;

    private static native SeqList getSequences0(long h, double mass, double tol) throws DBIndexStoreException;

    private static native SeqList getSequencesRanges0(long h, double[] mass, double[] tol)
            throws DBIndexStoreException;

    static native SeqList cutAndSearch0(long h, double[] mass, double[] tol) throws DBIndexStoreException;

    private static native long addProteinDef0(long h, long num, String def, String seq)
            throws DBIndexStoreException;

    private static native long getNumberSequences0(long h) throws DBIndexStoreException;

    private static native long getTotalSeqCount0(long h) throws DBIndexStoreException;

    private static native int[] getEntryKeys0(long h) throws DBIndexStoreException;

    private static native String proteinDef0(long h, long id) throws DBIndexStoreException;

    private static native String proteinSequence0(long h, long id) throws DBIndexStoreException;

    private static native void setDeviceDigest0(long h, boolean on) throws DBIndexStoreException;

    private static native void setPersist0(long h, boolean on) throws DBIndexStoreException;

    private static native void setUnindexed0(long h, int mode) throws DBIndexStoreException;
}
