package edu.scripps.yates.dbindex.hip;

import java.io.IOException;

import edu.scripps.yates.dbindex.DBIndexer;
import edu.scripps.yates.utilities.fasta.dbindex.DBIndexSearchParams;
import edu.scripps.yates.utilities.fasta.dbindex.DBIndexStoreException;

/**
 * {@link DBIndexer} whose protected {@code cutSeq} (DBIndexer.java:237) only
 * hands each protein to the store: the cutSeq loop itself runs on the GPU
 * inside {@link DBIndexStoreHip#stopAddSeq()}, so no per-peptide JNI call
 * happens.  Everything else — init(), run() (FASTA order, protein ids,
 * indexExists reuse), getSequencesUsingDaltonTolerance / PPMTolerance,
 * getProteins(String) — is the reference's own code.
 *
 * Usage: {@code new DBIndexerHip(params, IndexerMode.INDEX, new DBIndexStoreHip(params, 0))}.
 */
public class DBIndexerHip extends DBIndexer {

    public DBIndexerHip(DBIndexSearchParams sparam, IndexerMode mode, DBIndexStoreHip store)
            throws DBIndexStoreException {
        super(sparam, mode, store);  // DBIndexer.java:143-155
        store.setDeviceDigest(true);
        if (mode == IndexerMode.SEARCH_UNINDEXED) {
            store.setUnindexed(1);  // DBI_UNINDEXED_RESIDENT
        }
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
