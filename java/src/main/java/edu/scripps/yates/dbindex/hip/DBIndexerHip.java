package edu.scripps.yates.dbindex.hip;

import java.io.IOException;
import java.util.ArrayList;
import java.util.List;

import edu.scripps.yates.dbindex.DBIndexer;
import edu.scripps.yates.dbindex.util.IndexUtil;
import edu.scripps.yates.utilities.fasta.dbindex.DBIndexSearchParams;
import edu.scripps.yates.utilities.fasta.dbindex.DBIndexStoreException;
import edu.scripps.yates.utilities.fasta.dbindex.IndexedSequence;
import edu.scripps.yates.utilities.fasta.dbindex.MassRange;

/**
 * {@link DBIndexer} whose protected {@code cutSeq} (DBIndexer.java:237) only
 * hands each protein to the store: the cutSeq loop itself runs on the GPU
 * inside {@link DBIndexStoreHip#stopAddSeq()}, so no per-peptide JNI call
 * happens.  Everything else — init(), run() (FASTA order, protein ids,
 * indexExists reuse), getSequencesUsingDaltonTolerance / PPMTolerance,
 * getProteins(String) — is the reference's own code.  In SEARCH_UNINDEXED
 * mode the three query entry points go to {@link DBIndexStoreHip#cutAndSearch}
 * instead of the reference's private cutAndSearch, whose
 * {@code (MassRangeFilteringIndex) indexStore} cast (DBIndexer.java:713) would
 * not hold for this store.
 *
 * Usage: {@code new DBIndexerHip(params, IndexerMode.INDEX, new DBIndexStoreHip(params, 0))}.
 */
public class DBIndexerHip extends DBIndexer {

    private final DBIndexStoreHip hipStore;
    private final boolean unindexed;

    public DBIndexerHip(DBIndexSearchParams sparam, IndexerMode mode, DBIndexStoreHip store)
            throws DBIndexStoreException {
        super(sparam, mode, store);  // DBIndexer.java:143-155
        hipStore = store;
        unindexed = mode == IndexerMode.SEARCH_UNINDEXED;
        store.setDeviceDigest(true);
        if (unindexed) {
            store.setUnindexed(1);  // DBI_UNINDEXED_RESIDENT
        }
    }

    @Override
    public List<IndexedSequence> getSequencesUsingDaltonTolerance(double precursorMass, double massToleranceInDa)
            throws DBIndexStoreException {                                         // :762-772
        if (!unindexed) {
            return super.getSequencesUsingDaltonTolerance(precursorMass, massToleranceInDa);
        }
        return hipStore.cutAndSearch(oneRange(precursorMass, massToleranceInDa));
    }

    @Override
    public List<IndexedSequence> getSequencesUsingPPMTolerance(double precursorMass, double massToleranceInPPM)
            throws DBIndexStoreException {                                         // :787-797
        if (!unindexed) {
            return super.getSequencesUsingPPMTolerance(precursorMass, massToleranceInPPM);
        }
        final double massTolerance = IndexUtil.getToleranceInDalton(precursorMass, massToleranceInPPM);
        return hipStore.cutAndSearch(oneRange(precursorMass, massTolerance));
    }

    @Override
    public List<IndexedSequence> getSequences(List<MassRange> massRanges) throws DBIndexStoreException {  // :855-860
        return unindexed ? hipStore.cutAndSearch(massRanges) : super.getSequences(massRanges);
    }

    private static List<MassRange> oneRange(double precursorMass, double tolerance) {
        final List<MassRange> ranges = new ArrayList<MassRange>(1);
        ranges.add(new MassRange(precursorMass, tolerance));
        return ranges;
    }

    @Override
    protected void cutSeq(final String protAccession, String protSeq) throws IOException {
        // inline [formula] PTMs (DBIndexer.java:288-303) go to the store as they
        // are: the engine strips them and walks their proteins as cutSeq does
        try {
            indexStore.addProteinDef(++protNum, protAccession, protSeq);  // as cutSeq does (:251)
        } catch (final Exception e) {
            throw new IOException(e);  // nothing swallowed (the reference logs and continues, :398-403)
        }
    }
}
