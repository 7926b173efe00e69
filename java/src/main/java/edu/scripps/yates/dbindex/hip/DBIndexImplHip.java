package edu.scripps.yates.dbindex.hip;

import edu.scripps.yates.dbindex.DBIndexImpl;
import edu.scripps.yates.dbindex.DBIndexer.IndexerMode;
import edu.scripps.yates.dbindex.DBIndexerException;
import edu.scripps.yates.dbindex.util.IndexUtil;
import edu.scripps.yates.utilities.fasta.dbindex.DBIndexSearchParams;
import edu.scripps.yates.utilities.fasta.dbindex.DBIndexStoreException;
import edu.scripps.yates.utilities.masses.AssignMass;

/**
 * {@link DBIndexImpl} whose indexer is {@link DBIndexerHip} over a persisted
 * {@link DBIndexStoreHip}: the constructor follows DBIndexImpl(sParam, mode)
 * (DBIndexImpl.java:117-145) — init() in the requested mode, and when that
 * fails (no index yet for SEARCH_INDEXED) a fresh INDEX-mode indexer that
 * init()s and run()s, i.e. builds the index on the GPU and persists it.  Every
 * other DBIndexInterface method is DBIndexImpl's own, delegating to the indexer.
 *
 * Usage: {@code DBIndexInterface dbIndex = new DBIndexImplHip(params, 0);}
 */
public class DBIndexImplHip extends DBIndexImpl {

    public DBIndexImplHip(DBIndexSearchParams sParam, int device) throws DBIndexStoreException {
        // DBIndexImpl(sParam) (:101-115): indexed when the params ask for an index
        this(sParam, sParam.isUseIndex() ? IndexerMode.SEARCH_INDEXED : IndexerMode.SEARCH_UNINDEXED, device);
    }

    public DBIndexImplHip(DBIndexSearchParams sParam, IndexerMode indexerMode, int device)
            throws DBIndexStoreException {
        super();
        AssignMass.getInstance(sParam.isUseMonoParent());                          // :121
        indexer = new DBIndexerHip(sParam, indexerMode, newStore(sParam, device));
        try {
            indexer.init();
        } catch (final DBIndexerException ex) {
            // no index on disk yet (:127-140): index now, on the GPU
            indexer = new DBIndexerHip(sParam, IndexerMode.INDEX, newStore(sParam, device));
            try {
                indexer.init();
                indexer.run();
            } catch (final DBIndexerException e) {
                throw new DBIndexStoreException("Could not index the database: " + e.getMessage());
            }
        }
        dbIndexByParamKey.put(IndexUtil.createFullIndexFileName(sParam), this);    // :144
    }

    private static DBIndexStoreHip newStore(DBIndexSearchParams sParam, int device) throws DBIndexStoreException {
        final DBIndexStoreHip store = new DBIndexStoreHip(sParam, device);
        store.setPersist(true);  // indexExists() across processes (DBIndexer.java:522-527)
        return store;
    }
}
